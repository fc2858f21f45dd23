#!/bin/bash
# quick GPU check: gpu tests, GEMM microbench, BERT + ResNet bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-quick}
mkdir -p $OUT
fatal() { case $1 in 0|1|2) return 0;; *) echo "step $2 rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log; tail -3 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 300 python scripts/bench_gemm.py > $OUT/gemm.log 2>&1; rc=$?; cat $OUT/gemm.log; fatal $rc gemm
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert_native.log 2>&1; rc=$?
tail -1 $OUT/bert_native.log; fatal $rc bert
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/resnet_native.log 2>&1; rc=$?
tail -1 $OUT/resnet_native.log; fatal $rc resnet
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bert -- python bench.py --model bert-base --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
