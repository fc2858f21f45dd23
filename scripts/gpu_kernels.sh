#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/k1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/k1/pytest.log 2>&1 &&
timeout -k 10 400 python scripts/bench_conv.py --batch 256 --iters 10 --json gpurun_out/k1/conv.json > gpurun_out/k1/conv.log 2>&1
echo "exit $?"
