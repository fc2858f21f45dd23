#!/bin/bash
# Stock PyTorch-ROCm baseline for the headline bench + kernel profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/baseline
timeout -k 10 120 python -c "import torch;p=torch.cuda.get_device_properties(0);print(p);print(torch.version.hip)" > gpurun_out/baseline/devinfo.txt 2>&1 &&
timeout -k 10 400 python bench.py --impl torch --steps 20 --warmup 8 > gpurun_out/baseline/bench_torch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/baseline/prof -o torch -- python bench.py --impl torch --steps 5 --warmup 5 > gpurun_out/baseline/prof.log 2>&1
echo "exit $?"
