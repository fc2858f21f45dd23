#!/bin/bash
# Kernel trace of the captured training step (graph replay) per model + idle-gap analysis
# (scripts/step_gaps.py) and per-queue busy time (scripts/queue_busy.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-trace}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
for m in ${TRACE_MODELS:-bert-base resnet50}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$m -o k -- python bench.py --model $m --steps 4 --warmup 3 > $OUT/tr_$m.log 2>&1; rc=$?
  fatal $rc trace_$m
  mk=sgd_kernel; [ $m = unet ] && mk=adam; [ $m = bert-base ] && mk=adam
  python scripts/step_gaps.py $OUT/tr_$m/k_kernel_trace.csv $mk 20 > $OUT/gaps_$m.txt 2>&1; head -3 $OUT/gaps_$m.txt
  python scripts/queue_busy.py $OUT/tr_$m/k_kernel_trace.csv $mk > $OUT/queues_$m.txt 2>&1; cat $OUT/queues_$m.txt | head -40
done
