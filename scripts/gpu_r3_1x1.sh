#!/bin/bash
# round 3: ResNet-50 bench + 1x1-conv main-loop variants vs hipBLASLt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3a}
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 500 python scripts/bench_1x1.py > $OUT/b1x1.log 2>&1 || { echo "b1x1 rc=$?"; tail -20 $OUT/b1x1.log; exit 1; }
tail -2 $OUT/b1x1.log
