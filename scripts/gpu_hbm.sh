#!/bin/bash
# HBM traffic per kernel of the three benches: two rocprofv3 counter passes (FETCH_SIZE uses 3
# TCC counters, WRITE_SIZE 2, so they cannot share a pass), each with --kernel-trace only.
# scripts/hbm_table.py joins them per dispatch into achieved TB/s per kernel family.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-hbm}
mkdir -p $OUT
for m in ${HBM_MODELS:-resnet50 bert-base unet}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/${m}_$c -o k -- \
      python bench.py --model $m --steps 2 --warmup 1 --graph 0 > $OUT/${m}_$c.log 2>&1
    rc=$?; echo "$m $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
