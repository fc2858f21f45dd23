#!/bin/bash
# round-6 GPU pass 20: rows per thread (1 / 2 / 4) of the folded-finalize BN passes - isolated
# shapes and the ResNet-50 step, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bn_" > $O/pytest_k.log 2>&1 || exit $?
: > $O/shapes.jsonl
for u in 1 2 4; do
  MLC_BN_UNROLL=$u timeout -k 10 300 python -u scripts/bench_bn_fused.py | sed "s/^{/{\"unroll\": $u, /" >> $O/shapes.jsonl || exit $?
done
: > $O/ab.jsonl
for r in 1 2 3; do
  for v in "MLC_BN_UNROLL=1" "MLC_BN_UNROLL=2" "MLC_BN_UNROLL=4"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
tail -1 $O/pytest_k.log; python -c "
import json
for l in open('$O/shapes.jsonl'):
    d=json.loads(l); print(d['unroll'], d['shape'], d['fwd_us_fused'], d['bwd_us_fused'])
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['value'])"
