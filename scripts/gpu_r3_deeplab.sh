#!/bin/bash
# native DeepLab: seg GPU tests, DeepLab native vs stock bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3aa}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_seg_gpu.py tests/test_kernels_gpu.py -k "seg or bilinear or deeplab or pspnet or fpn or linknet or unet or upcat or bn_fwd_bwd" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for impl in native torch; do
  timeout -k 10 300 python bench.py --model deeplab --impl $impl --steps 20 --warmup 5 > $OUT/deeplab_$impl.log 2>&1 || { echo "bench $impl rc=$?"; tail -30 $OUT/deeplab_$impl.log; exit 1; }
  tail -1 $OUT/deeplab_$impl.log | cut -c1-200
done
