#!/bin/bash
# Generic-engine throughput table: every model native and on stock PyTorch-ROCm.
# Usage (on the GPU box): bash scripts/bench_generic_all.sh OUT_FILE [impl...]
set -o pipefail
OUT=${1:-gpurun_out/generic_bench.jsonl}; shift
mkdir -p "$(dirname "$OUT")"
IMPLS=${@:-native torch}
T=${STEP_TIMEOUT:-240}
run() {
  for impl in $IMPLS; do
    timeout -k 10 "$T" python -u scripts/bench_generic.py --impl "$impl" "$@" >> "$OUT" || return $?
  done
}
run --model LeNet --batch 256 --size 28 --channels 1 --classes 10 &&
run --model ref_cifar_net --batch 256 --size 32 --classes 10 &&
run --model resnext50_32x4d --batch 64 --size 224 &&
run --model se_resnext50_32x4d --batch 64 --size 224 &&
run --model efficientnet-b0 --batch 64 --size 224 &&
run --model unet:resnext50_32x4d --batch 16 --size 256 --classes 2 &&
run --model psp:resnet34 --batch 16 --size 256 --classes 21 &&
run --model deeplab:resnet --batch 8 --size 256 --classes 21 &&
run --model deeplab:mobilenet --batch 16 --size 256 --classes 21 &&
run --model linknet:resnet34 --batch 16 --size 256 --classes 2
