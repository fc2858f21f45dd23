#!/bin/bash
# round 3 end of session: full GPU test suite, stats-epilogue microbench, the three benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python scripts/bench_conv_stats.py > $OUT/conv_stats.jsonl 2>&1 || { echo "stats bench rc=$?"; tail -20 $OUT/conv_stats.jsonl; exit 1; }
tail -1 $OUT/conv_stats.jsonl
for m in resnet50 bert-base unet; do
  timeout -k 10 300 python bench.py --model $m > $OUT/bench_$m.log 2>&1 || { echo "bench $m rc=$?"; tail -20 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log | cut -c1-200
done
