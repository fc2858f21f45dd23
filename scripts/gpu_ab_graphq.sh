#!/bin/bash
# Interleaved A/B of the HIP graph executor's stream count (DEBUG_HIP_FORCE_GRAPH_QUEUES,
# "def" = unset) on the ResNet-50 / BERT-base / U-Net benches, plus one kernel trace per
# setting of interest (GRAPHQ_TRACE="2") for the cross-queue gap analysis.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-graphq}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
for model in ${AB_MODELS:-resnet50 bert-base unet}; do
  for i in 1 2; do
    for v in ${AB_VALUES:-def 1 2 4}; do
      if [ "$v" = def ]; then
        timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 > $OUT/${model}_${v}_$i.log 2>&1; rc=$?
      else
        DEBUG_HIP_FORCE_GRAPH_QUEUES=$v timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 > $OUT/${model}_${v}_$i.log 2>&1; rc=$?
      fi
      echo "$model Q=$v run $i: $(tail -1 $OUT/${model}_${v}_$i.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*')"; fatal $rc bench
    done
  done
done
for v in $GRAPHQ_TRACE; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_q$v -o k -- python bench.py --model resnet50 --steps 4 --warmup 3 > $OUT/tr_q$v.log 2>&1; rc=$?
  fatal $rc trace_q$v
  python scripts/step_gaps.py $OUT/tr_q$v/k_kernel_trace.csv sgd_kernel 10 > $OUT/gaps_q$v.txt 2>&1; head -3 $OUT/gaps_q$v.txt
done
