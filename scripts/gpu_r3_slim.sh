#!/bin/bash
# round 3: 256x32 tile numerics + U-Net / ResNet A/B (MLC_GEMM_SLIM)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3o}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_seg_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for sl in 0 1; do
    MLC_GEMM_SLIM=$sl timeout -k 10 300 python bench.py --model unet > $OUT/unet_s${sl}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/unet_s${sl}_$r.log; exit 1; }
    echo "slim=$sl r=$r $(grep -o '"value": [0-9.]*' $OUT/unet_s${sl}_$r.log)"
  done
done
