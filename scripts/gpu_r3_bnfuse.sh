#!/bin/bash
# round 3: ResNet-50 A/B of the BN-apply fusion into 1x1 consumers (MLC_FUSE_BN_FWD 0 / 3 / 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3g}
mkdir -p $OUT
for r in 1 2; do
  for m in 0 3 1; do
    MLC_FUSE_BN_FWD=$m timeout -k 10 300 python bench.py > $OUT/r50_f${m}_$r.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/r50_f${m}_$r.log; exit 1; }
    echo "fuse=$m r=$r $(grep -o '"value": [0-9.]*' $OUT/r50_f${m}_$r.log)"
  done
done
