#!/bin/bash
# Re-check of the stream knobs on the final kernels: U-Net shortcut stream, ResNet per-block joins
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-streams}; mkdir -p $OUT
run() { local label=$1; shift; env "$@" timeout -k 10 300 python bench.py $BENCH_ARGS > $OUT/$label.log 2>&1 || { echo "$label failed"; exit 1; }
  echo "$label: $(tail -1 $OUT/$label.log | cut -c60-100)"; }
BENCH_ARGS="--model unet --steps 30 --warmup 5"
run unet_base MLC_X=0; run unet_down MLC_DOWN_STREAM_UNET=1; run unet_base2 MLC_X=0; run unet_down2 MLC_DOWN_STREAM_UNET=1
BENCH_ARGS=""
run rn_base MLC_X=0; run rn_ws2 MLC_WGRAD_STREAM=2; run rn_base2 MLC_X=0; run rn_ws2b MLC_WGRAD_STREAM=2
