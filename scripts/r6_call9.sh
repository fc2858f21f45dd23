#!/bin/bash
# round-6 GPU pass 9: correctness anchor at the fp32-ulp noise floor; stock PyTorch's own
# GPU-vs-CPU floor; ResNet-50 headline with the BN block cap at 512
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i
mkdir -p $O
MLC_DETERMINISTIC=1 timeout -k 10 900 python -u scripts/engines_det_compare.py --noise \
  resnet50 bert resnext50 unet linknet fpn pspnet deeplab efficientnet-b0 unet-resnext50 \
  > $O/engines_det.jsonl 2> $O/engines_det.err || exit $?
timeout -k 10 600 python -u scripts/torch_cross_device.py > $O/torch_cross.jsonl 2> $O/torch_cross.err || exit $?
: > $O/bench.jsonl
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
python - <<'PY'
import json
for l in open('gpurun_out/r6i/engines_det.jsonl'):
    d = json.loads(l)
    print(d['kind'], 'gpu med %.3g max %.3g | noise med %.3g max %.3g | ratio med %.2f slotmax %.2f' % (
        d['grad_rel_median'], d['grad_rel_max'], d['noise_median'], d['noise_max'], d['ratio_median'], d['ratio_slot_max']))
for l in open('gpurun_out/r6i/torch_cross.jsonl'):
    d = json.loads(l)
    print(d['model'], 'torch gpu-vs-cpu med %.3g max %.3g | noise med %.3g max %.3g' % (
        d['gpu_vs_cpu_median'], d['gpu_vs_cpu_max'], d['cpu_fp32ulp_noise_median'], d['cpu_fp32ulp_noise_max']))
for l in open('gpurun_out/r6i/bench.jsonl'):
    print(json.loads(l)['value'])
PY
