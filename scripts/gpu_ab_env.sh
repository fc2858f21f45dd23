#!/bin/bash
# Generic interleaved A/B of an environment knob on the three benches:
#   AB_VAR=MLC_OPT_IN_BWD AB_VALUES="1 0" bash scripts/gpu_ab_env.sh
# plus the GPU tests first (stop on a crash).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-ab}
mkdir -p $OUT
fatal() { case $1 in 0|1) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  tail -2 $OUT/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || exit 1
fi
for model in ${AB_MODELS:-resnet50 bert-base unet}; do
  for i in 1 2; do
    for v in $AB_VALUES; do
      env $AB_VAR=$v timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 $AB_ARGS > $OUT/${model}_${v##*/}_$i.log 2>&1; rc=$?
      echo "$model $AB_VAR=$v run $i: $(tail -1 $OUT/${model}_${v##*/}_$i.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*')"; fatal $rc bench
    done
  done
done
