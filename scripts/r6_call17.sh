#!/bin/bash
# round-6 GPU pass 17: block-per-bin adaptive pool (PSPNet), profiles of the generic zoo models
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_seg_gpu.py -k "adaptive or psp or stats_into" > $O/pytest_k.log 2>&1 || exit $?
: > $O/bench.jsonl
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model pspnet --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
for m in efficientnet-b0:256:224 se_resnext50_32x4d:64:224 densenet121:64:224; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o $name -- python scripts/bench_generic.py --model $name --batch $b --size $sz --steps 6 --warmup 3 > $O/prof_$name.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o pspnet -- python bench.py --model pspnet --steps 6 --warmup 3 > $O/prof_psp.log 2>&1 || exit $?
tail -1 $O/pytest_k.log; python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['config']['model'], d['value'])"
