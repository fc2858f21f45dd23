#!/bin/bash
# round-6 GPU pass 4: graph / NULL-stream bisection (stock PyTorch only) + dense weight-gradient
# reduction A/B (atomics vs slabs) on BERT-base and ViT-B/16, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d
mkdir -p $O
: > $O/graph_bisect.jsonl
for m in conv bn effnet mlp; do
  for mode in null estream noeager evalnull sharedpool; do
    timeout -k 10 120 python -u scripts/graph_null_stream_bisect.py $m $mode >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
  done
  PYTORCH_NO_HIP_MEMORY_CACHING=1 timeout -k 10 120 python -u scripts/graph_null_stream_bisect.py $m nocache >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
done
: > $O/wgrad_ab.jsonl
for r in 1 2; do
  for v in slab atomic; do
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"bert-base\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
    MLC_DENSE_WGRAD=$v timeout -k 10 300 python -u bench.py --model vit-b16 --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"model\": \"vit-b16\", \"dense_wgrad\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/wgrad_ab.jsonl
  done
done
cat $O/graph_bisect.jsonl; python -c "
import json
for l in open('$O/wgrad_ab.jsonl'):
    d=json.loads(l); print(d['model'], d['dense_wgrad'], d['run'], d['line']['value'])"
