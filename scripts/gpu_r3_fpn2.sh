#!/bin/bash
# native bilinear upsampling for FPN: seg GPU tests, FPN bench, FPN kernel profile (summarised on the box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3x}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_seg_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --model fpn --steps 20 --warmup 5 > $OUT/fpn_native.log 2>&1 || { echo "bench rc=$?"; tail -30 $OUT/fpn_native.log; exit 1; }
tail -1 $OUT/fpn_native.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fpn -o run -- python bench.py --model fpn --steps 8 --warmup 3 > $OUT/prof_fpn.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_fpn.log; exit 1; }
python scripts/rocpd_stats.py $OUT/prof_fpn --steps 11 --top 45 > $OUT/kernels_fpn.txt 2>&1
rm -rf $OUT/prof_fpn
head -12 $OUT/kernels_fpn.txt | cut -c1-150
