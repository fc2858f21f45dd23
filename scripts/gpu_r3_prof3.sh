#!/bin/bash
# round 3 session 2: kernel-trace profiles of the BERT-base, ResNet-50, LinkNet and FPN steps,
# summarised on the box (the SQLite traces are too large to copy back)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3w}
mkdir -p $OUT
for m in bert-base resnet50 linknet fpn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 8 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
  python scripts/rocpd_stats.py $OUT/prof_$m --steps 11 --top 45 > $OUT/kernels_$m.txt 2>&1 || { echo "stats $m failed"; tail -5 $OUT/kernels_$m.txt; exit 1; }
  find $OUT/prof_$m -name "*kernel_stats.csv" -exec cp {} $OUT/${m}_kernel_stats.csv \;
  rm -rf $OUT/prof_$m
  head -3 $OUT/kernels_$m.txt
done
