#!/bin/bash
# round 3: stream-K numerics + per-shape A/B + ResNet-50 step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_streamk_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/sk_tests.log 2>&1 || { echo "sk tests rc=$?"; tail -30 $OUT/sk_tests.log; exit 1; }
tail -2 $OUT/sk_tests.log
timeout -k 10 400 python scripts/bench_sk.py > $OUT/bench_sk.log 2>&1 || { echo "bench_sk rc=$?"; tail -20 $OUT/bench_sk.log; exit 1; }
tail -1 $OUT/bench_sk.log
for sk in 0 90 0 90; do
  MLC_GEMM_SK=$sk timeout -k 10 300 python bench.py > $OUT/bench_sk$sk.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench_sk$sk.log; exit 1; }
  echo "sk=$sk $(tail -1 $OUT/bench_sk$sk.log | cut -c1-120)"
done
