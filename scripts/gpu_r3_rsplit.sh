#!/bin/bash
# ResNet-50 A/B of the conv weight-gradient split-K targets on the current kernels, plus the
# stock-PyTorch FPN line for the records
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3y}
mkdir -p $OUT
timeout -k 10 300 python bench.py --model fpn --impl torch --steps 20 --warmup 5 > $OUT/fpn_torch.log 2>&1 || { echo "fpn torch rc=$?"; tail -20 $OUT/fpn_torch.log; exit 1; }
for r in 1 2; do
  for cfg in "384 128" "256 128" "512 128" "384 64" "384 192"; do
    set -- $cfg
    MLC_SPLIT_TARGET=$1 MLC_SPLIT_TARGET_MAT=$2 timeout -k 10 300 python bench.py > $OUT/rn_${1}_${2}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/rn_${1}_${2}_$r.log; exit 1; }
    echo "split_target=$1 mat=$2 r=$r $(grep -o '"value": [0-9.]*' $OUT/rn_${1}_${2}_$r.log)"
  done
done
