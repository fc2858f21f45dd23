#!/bin/bash
# GPU check: kernel numerics + engine tests, smoke, conv bench, native headline bench
# (eager + graph) and a rocprofv3 kernel-stats profile.  Stops at the first step that
# crashed / timed out (plain test failures continue so the bench still runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r}
mkdir -p $OUT

fatal() {  # rc -> 0 when it is safe to keep using the GPU
    case $1 in 0|1|2) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac
}

timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log; tail -3 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -1 $OUT/smoke.log; fatal $rc smoke
if [ -z "$SKIP_CONV" ]; then
  timeout -k 10 300 python scripts/bench_conv.py --iters 10 > $OUT/conv.log 2>&1; rc=$?
  tail -1 $OUT/conv.log; fatal $rc conv
fi
timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5 --graph 0 > $OUT/bench_native_eager.log 2>&1 && tail -1 $OUT/bench_native_eager.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench_native.log 2>&1 && tail -1 $OUT/bench_native.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o native -- python bench.py --impl native --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
