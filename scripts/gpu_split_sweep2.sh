#!/bin/bash
# second split-K target sweep around the first one's best (gathered 384, plain 128)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-split2}
mkdir -p $OUT
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py > $OUT/$label.log 2>&1 || { echo "$label failed"; exit 1; }
  echo "$label: $(tail -1 $OUT/$label.log | cut -c60-100)"
}
run base1 MLC_X=0
run t384 MLC_SPLIT_TARGET=384
run t256 MLC_SPLIT_TARGET=256
run t512 MLC_SPLIT_TARGET=512
run t384m128 MLC_SPLIT_TARGET=384 MLC_SPLIT_TARGET_MAT=128
run t256m128 MLC_SPLIT_TARGET=256 MLC_SPLIT_TARGET_MAT=128
run base2 MLC_X=0
run t384b MLC_SPLIT_TARGET=384
for m in unet bert-base; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > $OUT/${m}_base.log 2>&1 || exit 1
  MLC_SPLIT_TARGET=384 timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > $OUT/${m}_t384.log 2>&1 || exit 1
  echo "$m base: $(tail -1 $OUT/${m}_base.log | cut -c60-100)  t384: $(tail -1 $OUT/${m}_t384.log | cut -c60-100)"
done
