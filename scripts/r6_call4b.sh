#!/bin/bash
# round-6 GPU pass 4b: graph / NULL-stream bisection (conv, bn, effnet; mlp ran in pass 4),
# native temporal unfold test, dense weight-gradient A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d
mkdir -p $O
for m in conv bn effnet; do
  for mode in null estream noeager evalnull sharedpool; do
    timeout -k 10 120 python -u scripts/graph_null_stream_bisect.py $m $mode >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
  done
done
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k temporal -x -v --timeout 120 --timeout-method thread > $O/pytest_temporal.log 2>&1 || exit $?
: > $O/wgrad_ab.jsonl
for r in 1 2; do
  for v in slab atomic; do
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"bert-base\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model vit-b16 --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"vit-b16\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
  done
done
tail -3 $O/pytest_temporal.log; cat $O/graph_bisect.jsonl | cut -c1-220; python -c "
import json
for l in open('$O/wgrad_ab.jsonl'):
    d=json.loads(l); print(d['model'], d['dense_wgrad'], d['run'], d['line']['value'])"
