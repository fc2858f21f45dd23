#!/bin/bash
# round-6 GPU pass 13: folded BN finalize, loads issued together - isolated timing per shape,
# numerics, ResNet-50 A/B (interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bn_" > $O/pytest_k.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bench_bn_fused.py > $O/bn_shapes.jsonl 2> $O/bn_shapes.err || exit $?
: > $O/ab.jsonl
for r in 1 2 3; do
  for v in "MLC_BN_FUSED=1" "MLC_BN_FUSED=0"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/ab.err || exit $?
    echo "{\"knob\": \"$v\", \"run\": $r, \"line\": $(tail -1 $O/b.json)}" >> $O/ab.jsonl
  done
done
tail -1 $O/pytest_k.log; cat $O/bn_shapes.jsonl; python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['knob'], d['run'], d['line']['value'])"
for m in densenet121:64:224 inceptionv3:80:299; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o $name -- python scripts/bench_generic.py --model $name --batch $b --size $sz --steps 6 --warmup 3 > $O/prof_$name.log 2>&1 || exit $?
done
