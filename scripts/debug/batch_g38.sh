#!/bin/bash
export RUN_TAG=${RUN_TAG:-g38}
O=gpurun_out/$RUN_TAG
mkdir -p $O
STEP_TIMEOUT=240 bash scripts/bench_generic_all.sh $O/native.jsonl native || exit 1
STEP_TIMEOUT=240 bash scripts/bench_generic_all.sh $O/torch.jsonl torch || exit 1
for m in resnext50_32x4d efficientnet-b0; do
  STEPS=5 STEP_TIMEOUT=300 bash scripts/gpu.sh prof $m -- python3 scripts/bench_generic.py --model $m --batch 64 --size 224 --steps 5 --warmup 3 || exit 1
done
