#!/bin/bash
# LDS-DMA GEMM main loop (MLC_GEMM_DMA=0/1): numerics tests, per-shape conv timing, then
# ResNet-50 / U-Net / BERT-base step A/B, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-dma}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma" > $OUT/pytest_dma.log 2>&1; rc=$?
tail -2 $OUT/pytest_dma.log; fatal $rc pytest_dma
for v in 0 1; do
  MLC_GEMM_DMA=$v timeout -k 10 300 python -u scripts/bench_convs.py --torch 0 > $OUT/convs_dma$v.txt 2>&1; rc=$?
  tail -n 2 $OUT/convs_dma$v.txt; fatal $rc convs
done
for i in 1 2; do
  for v in 0 1; do
    MLC_GEMM_DMA=$v timeout -k 10 300 python bench.py > $OUT/resnet_dma${v}_$i.log 2>&1; rc=$?
    echo "resnet dma=$v run $i: $(tail -1 $OUT/resnet_dma${v}_$i.log | cut -c60-130)"; fatal $rc resnet
  done
done
for v in 0 1; do
  MLC_GEMM_DMA=$v timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/unet_dma${v}.log 2>&1; rc=$?
  echo "unet dma=$v: $(tail -1 $OUT/unet_dma${v}.log | cut -c60-140)"; fatal $rc unet
  MLC_GEMM_DMA=$v timeout -k 10 300 python bench.py --model bert-base --steps 30 --warmup 5 > $OUT/bert_dma${v}.log 2>&1; rc=$?
  echo "bert dma=$v: $(tail -1 $OUT/bert_dma${v}.log | cut -c60-140)"; fatal $rc bert
done
