#!/bin/bash
# round-6 GPU pass 6: graph / NULL-stream bisection round 2 (depthwise / SiLU / SE), persistent
# GEMM test on shapes that take it, BERT split-K in-kernel reduction A/B, video models
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f
mkdir -p $O
for m in dw silu se; do
  for mode in null evalnull estream; do
    timeout -k 10 120 python -u scripts/graph_null_stream_bisect.py $m $mode >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
  done
done
echo "bisect done"
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "persistent or temporal" -x -v --timeout 100 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
: > $O/splitk_ab.jsonl
for r in 1 2; do
  for v in 0 512; do
    MLC_SPLITK_FUSED=$v timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"bert-base\", \"splitk_fused_kb\": $v, \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/splitk_ab.jsonl
  done
done
echo "ab done"
for m in r2plus1d_18 resnext3d_18; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model video:$m --batch 16 --size 112 --frames 8 --classes 400 --impl native >> $O/video.jsonl 2>> $O/video.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o r3d -- python scripts/bench_generic.py --model video:resnext3d_18 --batch 16 --size 112 --frames 8 --classes 400 --impl native --steps 6 --warmup 3 > $O/prof_r3d.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_k.log; cut -c1-230 $O/graph_bisect.jsonl; cat $O/video.jsonl; python -c "
import json
for l in open('$O/splitk_ab.jsonl'):
    d=json.loads(l); print(d['model'], d['splitk_fused_kb'], d['run'], d['line']['value'])"
