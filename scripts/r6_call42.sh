#!/bin/bash
# round-6 GPU pass 42: depthwise input-gradient block cap, MLC_DW_DGRAD_CAP 8192 / 4096 / 2048
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n2
mkdir -p $O
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_DW_DGRAD_CAP=8192" "MLC_DW_DGRAD_CAP=4096" "MLC_DW_DGRAD_CAP=2048"; do
    env $v timeout -k 10 300 python -u scripts/bench_generic.py --model efficientnet-b0 --batch 256 --size 224 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['model'], d['line']['img_per_s'])"
