#!/bin/bash
# Round 3: determinism test + transformer tests after the MatMCSum change, then the
# BERT GEMM shapes native vs hipBLASLt with the default tile policy and with wide tiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3gemm}
mkdir -p $OUT
fatal() { case $1 in 0|1) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_deterministic_gpu.py tests/test_transformer_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
for big in 0 1; do
  MLC_GEMM_BIG=$big timeout -k 10 300 python scripts/bench_blas_vs_native.py > $OUT/blas_big$big.log 2>&1; rc=$?
  echo "big=$big rc=$rc"; fatal $rc blas$big
done
