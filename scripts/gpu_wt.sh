#!/bin/bash
# Transposed-filter dgrad: kernel tests, per-shape A/B, ResNet-50 / U-Net step A/B
# (MLC_DGRAD_WT=0/1, alternating), then the whole GPU test-suite.  Stops at the first
# step that crashed / timed out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-wt}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "transposed or wt_table or dgrad" > $OUT/pytest_wt.log 2>&1; rc=$?; tail -2 $OUT/pytest_wt.log; fatal $rc pytest_wt
timeout -k 10 300 python -u scripts/bench_dgrad_wt.py > $OUT/bench_dgrad_wt.txt 2>&1; rc=$?; tail -3 $OUT/bench_dgrad_wt.txt; fatal $rc bench_dgrad_wt
for i in 1 2; do
  for v in 0 1; do
    MLC_DGRAD_WT=$v timeout -k 10 300 python bench.py > $OUT/resnet_wt${v}_$i.log 2>&1; rc=$?
    echo "resnet wt=$v run $i: $(tail -1 $OUT/resnet_wt${v}_$i.log | cut -c1-140)"; fatal $rc resnet
  done
done
for v in 0 1; do
  MLC_DGRAD_WT=$v timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/unet_wt${v}.log 2>&1; rc=$?
  echo "unet wt=$v: $(tail -1 $OUT/unet_wt${v}.log | cut -c1-140)"; fatal $rc unet
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -1 $OUT/smoke.log; fatal $rc smoke
