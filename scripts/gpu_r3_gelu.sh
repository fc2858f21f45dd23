#!/bin/bash
# round 3: dense-epilogue numerics + BERT-base A/B of the stored GELU derivative (interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for gd in 0 1; do
    MLC_GELU_DERIV=$gd timeout -k 10 300 python bench.py --model bert-base > $OUT/bert_gd${gd}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bert_gd${gd}_$r.log; exit 1; }
    echo "gelu_deriv=$gd r=$r $(grep -o '"value": [0-9.]*' $OUT/bert_gd${gd}_$r.log)"
  done
done
