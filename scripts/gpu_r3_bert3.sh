#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3k}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for d in 0 1; do
    MLC_LN_DEFER=$d timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_d${d}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_d${d}_$r.log; exit 1; }
    echo "ln_defer=$d r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_d${d}_$r.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof.log; exit 1; }
