#!/bin/bash
# BN-apply loader fusion: kernel/engine tests, then an A/B of the ResNet-50 bench with the
# fusion on and off (alternating runs in one box call) and a kernel profile of the fused step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-bnfuse}
mkdir -p $OUT
fatal() { case $1 in 0|1) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "native_fused or bn_input" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for f in 0 1 2; do
    MLC_FUSE_BN_FWD=$f timeout -k 10 200 python bench.py --steps 30 --warmup 10 > $OUT/bench_f${f}_$i.log 2>&1; rc=$?
    echo "fuse=$f run $i: $(tail -1 $OUT/bench_f${f}_$i.log | cut -c1-150)"; fatal $rc bench
  done
done
MLC_FUSE_BN_FWD=1 timeout -k 10 200 python bench.py --model unet --steps 30 --warmup 5 > $OUT/bench_unet.log 2>&1; rc=$?; tail -1 $OUT/bench_unet.log | cut -c1-150; fatal $rc unet
MLC_FUSE_BN_FWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1; echo "prof rc=$?"
