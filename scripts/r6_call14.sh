#!/bin/bash
# round-6 GPU pass 14: branch-point gradient accumulation (Inception), fused BN default on -
# generic / zoo / pooling tests, Inception + DenseNet + ResNet-50 benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_generic_gpu.py tests/test_gate_gpu.py tests/test_kernels_gpu.py -k "not persistent" > $O/pytest_g.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_zoo_gpu.py > $O/pytest_zoo.log 2>&1 || exit $?
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
tail -1 $O/pytest_g.log; tail -1 $O/pytest_zoo.log; cut -c1-200 $O/bench.jsonl
