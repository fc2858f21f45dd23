#!/bin/bash
# round-6 GPU pass 18: relaxed folded-BN slices, DenseNet totals / DenseCat, GPU numerics of the
# generic engine (incl. DenseNet / Inception), zoo benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_generic_gpu.py tests/test_gate_gpu.py tests/test_seg_gpu.py -k "bn or generic or gate or strided or stats or adaptive or seg" > $O/pytest_g.log 2>&1 || exit $?
: > $O/generic.jsonl
for m in densenet121:64:224 efficientnet-b0:256:224 inceptionv3:80:299 se_resnext50_32x4d:64:224 resnext50_32x4d:128:224 resnet50:512:224; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size $sz >> $O/generic.jsonl 2>> $O/generic.err || exit $?
done
: > $O/bench.jsonl
for m in resnet50 resnet50 unet deeplab; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o densenet121 -- python scripts/bench_generic.py --model densenet121 --batch 64 --size 224 --steps 6 --warmup 3 > $O/prof_dn.log 2>&1 || exit $?
tail -1 $O/pytest_g.log; cut -c1-150 $O/generic.jsonl; python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['config']['model'], d['value'])"
