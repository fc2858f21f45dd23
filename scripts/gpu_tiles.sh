#!/bin/bash
# wide-wave GEMM tiles: numerics (both tile policies), GEMM microbench, BERT/ResNet A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-tiles}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm.py > $OUT/gemm.log 2>&1; rc=$?; cat $OUT/gemm.log; [ $rc -eq 0 ] || exit $rc
for big in 0 1; do
  MLC_GEMM_BIG=$big timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert_big$big.log 2>&1 || exit $?
  tail -1 $OUT/bert_big$big.log | cut -c1-200
  MLC_GEMM_BIG=$big timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/resnet_big$big.log 2>&1 || exit $?
  tail -1 $OUT/resnet_big$big.log | cut -c1-200
done
echo "exit 0"
