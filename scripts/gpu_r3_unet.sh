#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3m}
mkdir -p $OUT
timeout -k 10 300 python bench.py --model unet > $OUT/unet.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/unet.log; exit 1; }
echo "unet $(grep -o '"value": [0-9.]*' $OUT/unet.log)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_unet -o run -- python bench.py --model unet --steps 8 --warmup 3 > $OUT/prof_unet.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_unet.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_r50 -o run -- python bench.py --steps 8 --warmup 3 > $OUT/prof_r50.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_r50.log; exit 1; }
