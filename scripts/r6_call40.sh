#!/bin/bash
# round-6 GPU pass 40: normact backward reduction 2 vs 4 chunks per iteration (MLC_NORMACT_RED_UNROLL),
# generic zoo interleaved, + normact tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o2
mkdir -p $O
MLC_NORMACT_RED_UNROLL=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_generic_gpu.py -k "bnact or leading_channels" > $O/pytest4.log 2>&1 || exit $?
tail -1 $O/pytest4.log
: > $O/ab.jsonl
for r in 1 2; do
  for v in "MLC_NORMACT_RED_UNROLL=2" "MLC_NORMACT_RED_UNROLL=4"; do
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
