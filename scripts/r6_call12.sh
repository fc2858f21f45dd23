#!/bin/bash
# round-6 GPU pass 12: BN finalize folded into the apply passes - numerics, ResNet-50 A/B
# (interleaved), steady-state dispatch count
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "bn_" > $O/pytest_k.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_engines_gpu_vs_cpu.py tests/test_seg_gpu.py > $O/pytest_engines.log 2>&1 || exit $?
: > $O/ab.jsonl
for r in 1 2 3; do
  for v in "MLC_BN_FUSED=1" "MLC_BN_FUSED=0"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50 -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_k.log $O/pytest_engines.log | tail -4; python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['value'])"
