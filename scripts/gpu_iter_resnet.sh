#!/bin/bash
# quick iteration: selected GPU tests (PYTEST_K), ResNet-50 bench, kernel-stats profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-it}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_native_gpu.py} -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 python bench.py --model bert-base --steps 30 --warmup 5 > $OUT/bench_bert.log 2>&1; rc=$?; tail -1 $OUT/bench_bert.log | cut -c1-140; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/bench_unet.log 2>&1; rc=$?; tail -1 $OUT/bench_unet.log | cut -c1-140; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "prof rc=$?"
