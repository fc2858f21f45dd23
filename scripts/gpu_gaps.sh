#!/bin/bash
# Idle-gap analysis of the captured ResNet-50 / U-Net steps (kernel trace with graph replay
# on), then the whole GPU test-suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-gaps}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
for m in resnet50 unet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$m -o k -- python bench.py --model $m --steps 4 --warmup 3 > $OUT/tr_$m.log 2>&1; rc=$?
  fatal $rc trace_$m
  f=$(find $OUT/tr_$m -name '*kernel_trace.csv' | head -1)
  mk=sgd_kernel; [ $m = unet ] && mk=adam
  python scripts/step_gaps.py "$f" $mk 20 > $OUT/gaps_$m.txt 2>&1; head -3 $OUT/gaps_$m.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
