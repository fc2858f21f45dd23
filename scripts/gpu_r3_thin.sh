#!/bin/bash
# round 3: 32x256 weight-gradient tile numerics + U-Net A/B (MLC_GEMM_THIN)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3p}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_seg_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for t in 0 1; do
    MLC_GEMM_THIN=$t timeout -k 10 300 python bench.py --model unet > $OUT/unet_t${t}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/unet_t${t}_$r.log; exit 1; }
    echo "thin=$t r=$r $(grep -o '"value": [0-9.]*' $OUT/unet_t${t}_$r.log)"
  done
done
