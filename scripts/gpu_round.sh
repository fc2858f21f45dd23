#!/bin/bash
# GPU check: kernel numerics, native engine tests, conv bench, native + torch headline bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r}
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; echo "pytest rc=$?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
timeout -k 10 300 python scripts/bench_conv.py --iters 10 > $OUT/conv.log 2>&1; tail -1 $OUT/conv.log
timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5 --graph 0 > $OUT/bench_native_eager.log 2>&1 && tail -1 $OUT/bench_native_eager.log &&
timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5 > $OUT/bench_native.log 2>&1 && tail -1 $OUT/bench_native.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o native -- python bench.py --impl native --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
