#!/bin/bash
# native U-Net: kernel numerics + step test, U-Net bench native vs torch, profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-seg}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_seg_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -12 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model unet --steps 20 --warmup 5 > $OUT/unet_native.log 2>&1 && tail -1 $OUT/unet_native.log &&
timeout -k 10 300 python bench.py --model unet --impl torch --steps 20 --warmup 5 > $OUT/unet_torch.log 2>&1 && tail -1 $OUT/unet_torch.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o unet -- python bench.py --model unet --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
