#!/bin/bash
# 128x64 dense tiles for 768-wide outputs (MLC_DENSE_NARROW=0/1): dense-GEMM tests, then
# BERT-base step A/B, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-narrow}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
MLC_DENSE_NARROW=1 timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_tx.log 2>&1; rc=$?
tail -2 $OUT/pytest_tx.log; fatal $rc pytest_tx
for i in 1 2; do
  for v in 0 1; do
    MLC_DENSE_NARROW=$v timeout -k 10 300 python bench.py --model bert-base --steps 40 --warmup 5 > $OUT/bert_n${v}_$i.log 2>&1; rc=$?
    echo "bert narrow=$v run $i: $(tail -1 $OUT/bert_n${v}_$i.log | cut -c60-140)"; fatal $rc bert
  done
done
