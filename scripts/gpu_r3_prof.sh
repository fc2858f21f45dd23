#!/bin/bash
# round 3: optimizer numerics, benches, and kernel-stat profiles of the three flagship steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3c}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sgd_adam" --timeout 120 --timeout-method thread > $OUT/opt_tests.log 2>&1 || { echo "opt tests rc=$?"; tail -30 $OUT/opt_tests.log; exit 1; }
tail -1 $OUT/opt_tests.log
for m in resnet50 bert-base unet; do
  timeout -k 10 300 python bench.py --model $m > $OUT/bench_$m.log 2>&1 || { echo "bench $m rc=$?"; tail -20 $OUT/bench_$m.log; exit 1; }
  echo "$m $(tail -1 $OUT/bench_$m.log | cut -c1-110)"
done
for m in bert-base resnet50; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 8 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | head
