#!/bin/bash
# round-6 GPU pass 5: graph / NULL-stream bisection (conv, bn, effnet), native temporal unfold,
# dense weight-gradient A/B, then the persistent short-K GEMM (correctness test, shape bench)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e
mkdir -p $O
for m in conv bn effnet; do
  for mode in null estream noeager evalnull sharedpool; do
    timeout -k 10 120 python -u scripts/graph_null_stream_bisect.py $m $mode >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
  done
done
echo "bisect done"
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k temporal -x -v --timeout 120 --timeout-method thread > $O/pytest_temporal.log 2>&1 || { tail -30 $O/pytest_temporal.log; exit 1; }
echo "temporal done"
: > $O/wgrad_ab.jsonl
for r in 1 2; do
  for v in slab atomic; do
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"bert-base\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model vit-b16 --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"vit-b16\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
  done
done
echo "ab done"
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k persistent -x -v --timeout 100 --timeout-method thread > $O/pytest_persist.log 2>&1 || { tail -30 $O/pytest_persist.log; exit 1; }
timeout -k 10 240 python -u scripts/bench_persist.py > $O/bench_persist.jsonl 2> $O/bench_persist.err || { tail -20 $O/bench_persist.err; exit 1; }
tail -3 $O/pytest_temporal.log $O/pytest_persist.log; cut -c1-200 $O/graph_bisect.jsonl; cat $O/bench_persist.jsonl; python -c "
import json
for l in open('$O/wgrad_ab.jsonl'):
    d=json.loads(l); print(d['model'], d['dense_wgrad'], d['run'], d['line']['value'])"
