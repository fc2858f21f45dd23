#!/bin/bash
# round-6 GPU pass 28: DenseNet growth convs written straight into the concat buffer (conv
# output row stride, in-place tail statistics): kernel + generic GPU tests, chain A/B, trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bnact or bn_stats or leading_channels or channel_slice or conv_fwd" > $O/pytest_k.log 2>&1 || exit $?
tail -1 $O/pytest_k.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_generic_gpu.py > $O/pytest_g.log 2>&1 || exit $?
tail -1 $O/pytest_g.log
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_DENSE_CHAIN=1" "MLC_DENSE_CHAIN=0"; do
    env $v timeout -k 10 300 python -u scripts/bench_generic.py --model densenet121 --batch 64 --size 224 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['model'], d['line']['img_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o densenet121 -- python scripts/bench_generic.py --model densenet121 --batch 64 --size 224 --steps 6 --warmup 3 > $O/prof_densenet.log 2>&1 || exit $?
