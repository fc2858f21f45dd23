#!/bin/bash
# Transposed dense weights for BERT's input gradients (MLC_DENSE_WT=0/1): transformer and
# native-BERT GPU tests, then the BERT-base step A/B, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-densewt}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_native_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
for i in 1 2; do
  for v in 0 1; do
    MLC_DENSE_WT=$v timeout -k 10 300 python bench.py --model bert-base --steps 40 --warmup 5 > $OUT/bert_wt${v}_$i.log 2>&1; rc=$?
    echo "bert wt=$v run $i: $(tail -1 $OUT/bert_wt${v}_$i.log | cut -c60-140)"; fatal $rc bert
  done
done
