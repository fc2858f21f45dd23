#!/bin/bash
# native PSPNet: seg GPU tests, PSPNet native vs stock bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3z}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_seg_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for impl in native torch; do
  timeout -k 10 300 python bench.py --model pspnet --impl $impl --steps 20 --warmup 5 > $OUT/psp_$impl.log 2>&1 || { echo "bench $impl rc=$?"; tail -30 $OUT/psp_$impl.log; exit 1; }
  tail -1 $OUT/psp_$impl.log | cut -c1-200
done
