#!/bin/bash
# dgrad-first capture order (MLC_DGRAD_FIRST): the GPU tests that cover the native engines
# and graphs, then an interleaved A/B on the three benches and a trace of the new order.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-dgf}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_graphed_gpu.py tests/test_transformer_gpu.py tests/test_deterministic_gpu.py tests/test_seg_gpu.py tests/test_native_eval_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
for model in resnet50 bert-base unet; do
  for i in 1 2; do
    for v in 0 1; do
      MLC_DGRAD_FIRST=$v timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 > $OUT/${model}_${v}_$i.log 2>&1; rc=$?
      echo "$model DGRAD_FIRST=$v run $i: $(tail -1 $OUT/${model}_${v}_$i.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*')"; fatal $rc bench
    done
  done
done
RUN_TAG=${RUN_TAG:-dgf}/tr bash scripts/gpu_trace_steps.sh > $OUT/trace.log 2>&1; fatal $? trace
grep -h "step span\|time with\|^queue" $OUT/trace.log
