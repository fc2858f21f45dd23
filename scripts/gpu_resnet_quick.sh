#!/bin/bash
# ResNet-50 quick loop: kernel numerics, native engine tests, bench, rocprof kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-rq}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/resnet.log 2>&1 && tail -1 $OUT/resnet.log | cut -c1-220 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o rn -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
