#!/bin/bash
# kernel-trace profiles of the native segmentation engines (summarised on the box), with a
# count of library (MIOpen / hipBLASLt / rocBLAS) kernels in each step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3ac}
mkdir -p $OUT
for m in unet linknet fpn pspnet deeplab; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 6 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
  python scripts/rocpd_stats.py $OUT/prof_$m --steps 9 --top 200 > $OUT/kernels_$m.txt 2>&1 || { echo "stats $m failed"; exit 1; }
  rm -rf $OUT/prof_$m
  echo "$m: $(head -1 $OUT/kernels_$m.txt); library kernels: $( (grep -ciE 'miopen|Cijk_|rocblas|naive_conv|igemm_fwd_gtc|igemm_bwd|igemm_wrw' $OUT/kernels_$m.txt || true) )"
done
