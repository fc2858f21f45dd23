#!/bin/bash
# round 3: native LinkNet (transposed conv on the dgrad GEMMs) - GPU tests + native vs stock bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3s}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_seg_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python bench.py --model linknet --steps 20 --warmup 5 > $OUT/linknet_native.log 2>&1 || { echo "bench rc=$?"; tail -30 $OUT/linknet_native.log; exit 1; }
tail -1 $OUT/linknet_native.log
timeout -k 10 300 python bench.py --model linknet --impl torch --steps 20 --warmup 5 > $OUT/linknet_torch.log 2>&1 || { echo "bench torch rc=$?"; tail -30 $OUT/linknet_torch.log; exit 1; }
tail -1 $OUT/linknet_torch.log
timeout -k 10 300 python bench.py --model unet --steps 20 --warmup 5 > $OUT/unet_native.log 2>&1 || { echo "bench unet rc=$?"; tail -30 $OUT/unet_native.log; exit 1; }
tail -1 $OUT/unet_native.log
