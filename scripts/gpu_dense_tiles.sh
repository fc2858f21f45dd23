#!/bin/bash
# Three-wide dense tiles: numerics + per-shape timing, the transformer GPU tests, then an
# interleaved BERT-base step A/B of MLC_DENSE_TILE (0 = old 128x128 path, unset = auto)
# x MLC_DENSE_WT (transposed weights for the input gradients).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-dt2}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u scripts/bench_dense_tiles.py > $OUT/tiles.log 2>&1; rc=$?; fatal $rc tiles
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
for i in 1 2; do
  for cfg in "0 0" "-1 0" "0 1" "-1 1"; do
    set -- $cfg
    if [ "$1" = "-1" ]; then unset MLC_DENSE_TILE; else export MLC_DENSE_TILE=$1; fi
    MLC_DENSE_WT=$2 timeout -k 10 200 python bench.py --model bert-base --steps 30 --warmup 10 > $OUT/bert_t$1_w$2_$i.log 2>&1; rc=$?
    echo "bert tile=$1 wt=$2 run $i: $(tail -1 $OUT/bert_t$1_w$2_$i.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*')"; fatal $rc bench
  done
done
unset MLC_DENSE_TILE
