#!/bin/bash
# round-6 GPU pass 39 (final tree): full GPU suite, smoke, generic zoo benches, ResNet-50 headline x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_full.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_full.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
: > $O/bench.jsonl
for m in densenet121:64:224 efficientnet-b0:256:224 inceptionv3:80:299 se_resnext50_32x4d:64:224 resnext50_32x4d:128:224; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size $sz > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
cut -c1-220 $O/bench.jsonl
