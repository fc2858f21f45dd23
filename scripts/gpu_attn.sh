#!/bin/bash
# fused attention: numerics tests, BERT tests, BERT bench + profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-attn}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert_native.log 2>&1 && tail -1 $OUT/bert_native.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bert -- python bench.py --model bert-base --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
