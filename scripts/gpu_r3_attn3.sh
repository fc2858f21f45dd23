#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3n}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q -k "attention or attn or native_bert" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/bench_bert_parts.py > $OUT/parts.log 2>&1 || { echo "parts rc=$?"; tail -20 $OUT/parts.log; exit 1; }
tail -1 $OUT/parts.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_$r.log; exit 1; }
  echo "bert r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_$r.log)"
done
timeout -k 10 300 python bench.py --model unet > $OUT/unet.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/unet.log; exit 1; }
echo "unet $(grep -o '"value": [0-9.]*' $OUT/unet.log)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_unet -o run -- python bench.py --model unet --steps 8 --warmup 3 > $OUT/prof_unet.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_unet.log; exit 1; }
