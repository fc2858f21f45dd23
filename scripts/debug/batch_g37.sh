#!/bin/bash
# kernel tests + trajectories + strip/cap A/B + torch bench table (one gpurun call)
export RUN_TAG=${RUN_TAG:-g37}
O=gpurun_out/$RUN_TAG
mkdir -p $O
STEP_TIMEOUT=300 bash scripts/gpu.sh run ktest -- python -u -m pytest tests/test_generic_gpu.py -k "depthwise or bnact" -q --timeout 120 || exit 1
MLC_TRAJ_OUT=$O/traj.jsonl STEP_TIMEOUT=400 bash scripts/gpu.sh run traj -- python -u -m pytest tests/test_seg_gpu.py -k trajectory -q --timeout 300
for v in 0 1; do
  cap=$([ $v = 0 ] && echo 1024 || echo 512)
  for m in efficientnet-b0 resnext50_32x4d; do
    MLC_DW_STRIPS=$v MLC_NORMACT_CAP=$cap timeout -k 10 200 python -u scripts/bench_generic.py --model $m --batch 64 --size 224 >> $O/ab.jsonl || exit 1
  done
done
STEP_TIMEOUT=240 bash scripts/bench_generic_all.sh $O/torch.jsonl torch
