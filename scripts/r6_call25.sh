#!/bin/bash
# round-6 GPU pass 25: generic-engine BN pass grid caps (MLC_NORMACT_CAP reduce /
# MLC_NORMACT_APPLY_CAP apply) on EfficientNet-b0 and DenseNet-121, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6x
mkdir -p $O
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_NORMACT_CAP=512" "MLC_NORMACT_CAP=1024" "MLC_NORMACT_CAP=2048" "MLC_NORMACT_APPLY_CAP=1024" "MLC_NORMACT_APPLY_CAP=512"; do
    for m in efficientnet-b0:256 densenet121:64; do
      IFS=: read name b <<< "$m"
      env $v timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size 224 > $O/b.json 2>> $O/ab.err || exit $?
      echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
    done
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['model'], d['line']['img_per_s'])"
