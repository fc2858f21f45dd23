#!/bin/bash
# ResNet-50 step under split-K target variants (weight gradients), after the LDS-DMA change
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-split}
mkdir -p $OUT
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py > $OUT/$label.log 2>&1 || { echo "$label failed"; exit 1; }
  echo "$label: $(tail -1 $OUT/$label.log | cut -c60-100)"
}
run base1 MLC_X=0
run t384 MLC_SPLIT_TARGET=384
run t1536 MLC_SPLIT_TARGET=1536
run m128 MLC_SPLIT_TARGET_MAT=128
run m512 MLC_SPLIT_TARGET_MAT=512
run base2 MLC_X=0
