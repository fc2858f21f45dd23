#!/bin/bash
# round-6 GPU pass 30: fast index division in the depthwise strip kernels, + MLC_DW_XCD A/B: numerics,
# EfficientNet-b0 A/B interleaved, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generic_gpu.py -k "depthwise or efficientnet or mobilenet" > $O/pytest_g.log 2>&1 || exit $?
tail -1 $O/pytest_g.log
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_DW_XCD=1" "MLC_DW_XCD=0"; do
    env $v timeout -k 10 300 python -u scripts/bench_generic.py --model efficientnet-b0 --batch 256 --size 224 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['model'], d['line']['img_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o effnet -- python scripts/bench_generic.py --model efficientnet-b0 --batch 256 --size 224 --steps 6 --warmup 3 > $O/prof_effnet.log 2>&1 || exit $?
