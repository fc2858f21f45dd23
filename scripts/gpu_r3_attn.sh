#!/bin/bash
# round 3: fused S=128 attention backward: numerics, parts bench, BERT A/B; ResNet BN-fusion A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3h}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/bench_bert_parts.py > $OUT/parts.log 2>&1 || { echo "parts rc=$?"; tail -20 $OUT/parts.log; exit 1; }
tail -1 $OUT/parts.log
for r in 1 2; do
  for b in 0 1; do
    MLC_ATTN_BWD128=$b timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_b${b}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_b${b}_$r.log; exit 1; }
    echo "bwd128=$b r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_b${b}_$r.log)"
  done
done
for r in 1 2; do
  for m in 0 3 1; do
    MLC_FUSE_BN_FWD=$m timeout -k 10 300 python bench.py > $OUT/r50_f${m}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/r50_f${m}_$r.log; exit 1; }
    echo "fuse=$m r=$r $(grep -o '"value": [0-9.]*' $OUT/r50_f${m}_$r.log)"
  done
done
