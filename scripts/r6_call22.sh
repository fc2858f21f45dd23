#!/bin/bash
# round-6 GPU pass 22 (final tree): full GPU suite on the current tree (incl. the fp32-ulp anchor), smoke,
# Inception / DenseNet benches + Inception trace, ResNet-50 headline x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_full.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
: > $O/bench.jsonl
for m in inceptionv3:80:299 densenet121:64:224; do
  IFS=: read name b sz <<< "$m"
  timeout -k 10 300 python -u scripts/bench_generic.py --model $name --batch $b --size $sz >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o inceptionv3 -- python scripts/bench_generic.py --model inceptionv3 --batch 80 --size 299 --steps 6 --warmup 3 > $O/prof_inc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50 -- python bench.py --steps 6 --warmup 3 > $O/prof_rn50.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_full.log | tail -2; tail -2 $O/smoke.log; cut -c1-200 $O/bench.jsonl
