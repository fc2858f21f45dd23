#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3l}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py -x -q -k "embed or native_bert" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_$r.log; exit 1; }
  echo "bert r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof.log; exit 1; }
