#!/bin/bash
# round-6 GPU pass 16: re-measure the README tables on the final tree (generic zoo, video,
# torch.nn transformers, segmentation engines, BERT) + generic GPU tests for the folded BN
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_generic_gpu.py tests/test_gate_gpu.py -k "bnact or generic or gate or video or resnext or efficient or inception or stats_into or dense" > $O/pytest_g.log 2>&1 || exit $?
: > $O/generic.jsonl
for m in resnet50:512:224 resnext50_32x4d:128:224 efficientnet-b0:256:224 se_resnext50_32x4d:64:224 densenet121:64:224 inceptionv3:80:299; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size $sz >> $O/generic.jsonl 2>> $O/generic.err || exit $?
done
for m in r2plus1d_18 resnext3d_18; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model video:$m --batch 16 --size 112 --frames 8 --classes 400 --impl native >> $O/generic.jsonl 2>> $O/generic.err || exit $?
done
: > $O/bench.jsonl
for m in bert-base transformer-base vit-b16 unet linknet fpn pspnet deeplab resnet50 resnet50; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
tail -1 $O/pytest_g.log; cut -c1-160 $O/generic.jsonl; python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['config']['model'], d['value'], d['unit'], d['ms_per_step'])"
