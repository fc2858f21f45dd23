#!/bin/bash
# round 3: BERT-base A/B of the transposed dense-weight dgrads (MLC_DENSE_WT), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3d}
mkdir -p $OUT
for r in 1 2; do
  for wt in 0 1; do
    MLC_DENSE_WT=$wt timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_wt${wt}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_wt${wt}_$r.log; exit 1; }
    echo "wt=$wt r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_wt${wt}_$r.log)"
  done
done
MLC_DENSE_WT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_wt1 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > $OUT/prof_wt1.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_wt1.log; exit 1; }
