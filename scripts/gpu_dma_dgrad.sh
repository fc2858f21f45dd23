#!/bin/bash
# LDS-DMA copies for the strided-dgrad loaders (ConvDgradA x ConvDgradBT): numerics, the
# per-shape dgrad table (plain vs transposed filter), and the ResNet-50 / U-Net steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-dmadg}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma or transposed or dgrad" > $OUT/pytest_dg.log 2>&1; rc=$?
tail -2 $OUT/pytest_dg.log; fatal $rc pytest_dg
timeout -k 10 300 python -u scripts/bench_dgrad_wt.py > $OUT/bench_dgrad_wt.txt 2>&1; rc=$?; tail -n 1 $OUT/bench_dgrad_wt.txt; fatal $rc bench_dgrad_wt
for i in 1 2; do
  timeout -k 10 300 python bench.py > $OUT/resnet_$i.log 2>&1; rc=$?
  echo "resnet run $i: $(tail -1 $OUT/resnet_$i.log | cut -c60-130)"; fatal $rc resnet
done
timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/unet.log 2>&1; rc=$?
echo "unet: $(tail -1 $OUT/unet.log | cut -c60-140)"; fatal $rc unet
