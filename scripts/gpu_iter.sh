#!/bin/bash
# kernel iteration: gpu tests, conv shapes (+ wgrad split sweep), ResNet + BERT bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-iter}
mkdir -p $OUT
fatal() { case $1 in 0|1|2) return 0;; *) echo "step $2 rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log; tail -3 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 400 python scripts/bench_convs.py --torch 0 ${CONV_ARGS:-} > $OUT/convs.log 2>&1; rc=$?
cat $OUT/convs.log | grep -v amdgpu.ids; fatal $rc convs
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/resnet_native.log 2>&1; rc=$?
tail -1 $OUT/resnet_native.log; fatal $rc resnet
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert_native.log 2>&1; rc=$?
tail -1 $OUT/bert_native.log; fatal $rc bert
