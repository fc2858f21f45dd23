#!/bin/bash
# capture order (MLC_DGRAD_FIRST 0/1) on the LinkNet / FPN / PSPNet / DeepLab engines, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3ad}
mkdir -p $OUT
for r in 1 2; do
  for m in linknet fpn pspnet deeplab; do
    for d in 1 0; do
      MLC_DGRAD_FIRST=$d timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 8 > $OUT/${m}_${d}_${r}.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/${m}_${d}_${r}.log; exit 1; }
      echo "$m dgrad_first=$d r=$r $(tail -1 $OUT/${m}_${d}_${r}.log | grep -o '"value": [0-9.]*')"
    done
  done
done
