#!/bin/bash
# round-6 GPU pass 19: per-shape ResNet-50 conv table at 512 (native vs MIOpen), BERT trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 600 python -u scripts/bench_convs.py --batch 512 --iters 10 > $O/conv_shapes_b512.txt 2> $O/conv_shapes.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o bert -- python bench.py --model bert-base --steps 6 --warmup 3 > $O/prof_bert.log 2>&1 || exit $?
cat $O/conv_shapes_b512.txt
