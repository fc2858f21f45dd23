#!/bin/bash
# Lagged weight-gradient joins (MLC_WGRAD_LAG=0/1): correctness tests with the lag on, then
# ResNet-50 / U-Net step A/B, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-lag}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
MLC_WGRAD_LAG=1 timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py tests/test_dp_gpu.py tests/test_seg_gpu.py tests/test_graphed_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lag.log 2>&1; rc=$?
tail -2 $OUT/pytest_lag.log; fatal $rc pytest_lag
for i in 1 2; do
  for v in 0 1; do
    MLC_WGRAD_LAG=$v timeout -k 10 300 python bench.py > $OUT/resnet_lag${v}_$i.log 2>&1; rc=$?
    echo "resnet lag=$v run $i: $(tail -1 $OUT/resnet_lag${v}_$i.log | cut -c60-130)"; fatal $rc resnet
  done
done
for v in 0 1; do
  MLC_WGRAD_LAG=$v timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/unet_lag${v}.log 2>&1; rc=$?
  echo "unet lag=$v: $(tail -1 $OUT/unet_lag${v}.log | cut -c60-140)"; fatal $rc unet
done
