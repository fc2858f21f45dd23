#!/bin/bash
export RUN_TAG=${RUN_TAG:-g39}
O=gpurun_out/$RUN_TAG
mkdir -p $O
STEP_TIMEOUT=600 bash scripts/gpu.sh tests tests/test_generic_gpu.py || exit 1
for m in resnext50_32x4d efficientnet-b0 se_resnext50_32x4d; do
  timeout -k 10 200 python -u scripts/bench_generic.py --model $m --batch 64 --size 224 >> $O/ab.jsonl || exit 1
done
STEPS=5 STEP_TIMEOUT=300 bash scripts/gpu.sh prof resnext50_32x4d -- python3 scripts/bench_generic.py --model resnext50_32x4d --batch 64 --size 224 --steps 5 --warmup 3
