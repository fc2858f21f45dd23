#!/bin/bash
# round-6 GPU pass 8: BN elementwise-pass knobs on the ResNet-50 headline, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h
mkdir -p $O
: > $O/bn_knobs.jsonl
for r in 1 2 3; do
  for v in "" "MLC_BN_UNROLL=2" "MLC_BN_UNROLL=4" "MLC_BN_BLOCKS=1536" "MLC_BN_BLOCKS=512"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"${v:-default}\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/bn_knobs.jsonl
  done
done
python -c "
import json
for l in open('$O/bn_knobs.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['value'])"
