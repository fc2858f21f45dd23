#!/bin/bash
# round 3: BERT-base A/B of the bf16 dense-GEMM split-K target (MLC_DENSE_SPLIT_TARGET) and
# the dense weight-gradient split target (MLC_SPLIT_TARGET_DENSE)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3q}
mkdir -p $OUT
for r in 1 2; do
  for t in 384 0 192 768; do
    MLC_DENSE_SPLIT_TARGET=$t timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_t${t}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_t${t}_$r.log; exit 1; }
    echo "dense_split_target=$t r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_t${t}_$r.log)"
  done
  for t in 384 512; do
    MLC_SPLIT_TARGET_DENSE=$t timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_w${t}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_w${t}_$r.log; exit 1; }
    echo "wgrad_split_target=$t r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_w${t}_$r.log)"
  done
done
