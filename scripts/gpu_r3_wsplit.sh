#!/bin/bash
# round 3: BERT-base A/B of the dense weight-gradient split target (MLC_SPLIT_TARGET_DENSE)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3r}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q -k "dense or native_bert" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for t in 256 128 64; do
    MLC_SPLIT_TARGET_DENSE=$t timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_w${t}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_w${t}_$r.log; exit 1; }
    echo "wgrad_split_target=$t r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_w${t}_$r.log)"
  done
done
