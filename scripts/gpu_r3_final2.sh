#!/bin/bash
# round 3 end of session 2: full GPU test suite, smoke(), the three flagship benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3ab}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for m in resnet50 bert-base unet fpn; do
  timeout -k 10 300 python bench.py --model $m > $OUT/bench_$m.log 2>&1 || { echo "bench $m rc=$?"; tail -20 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log | cut -c1-160
done
