#!/bin/bash
# round-6 GPU pass 34: block cap of the one-call normact backward's reduction (MLC_NORMACT_BWD_CAP
# 512 / 1024 / 2048, no atomics there) on the generic zoo, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s
mkdir -p $O
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_NORMACT_BWD_CAP=512" "MLC_NORMACT_BWD_CAP=1024" "MLC_NORMACT_BWD_CAP=2048"; do
    for m in efficientnet-b0:256:224 densenet121:64:224 se_resnext50_32x4d:64:224 resnext50_32x4d:128:224; do
      IFS=: read name b sz <<< "$m"
      env $v timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size $sz > $O/b.json 2>> $O/ab.err || exit $?
      echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
    done
  done
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['model'], d['line']['img_per_s'])"
