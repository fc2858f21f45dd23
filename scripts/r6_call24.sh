#!/bin/bash
# round-6 GPU pass 24: block cap of the folded-finalize BN passes (ResNet-50, interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w
mkdir -p $O
: > $O/ab.jsonl
for r in 1 2 3; do
  for v in "MLC_BN_BLOCKS=512" "MLC_BN_BLOCKS=384" "MLC_BN_BLOCKS=256" "MLC_BN_BLOCKS=768"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['value'])"
