#!/bin/bash
# round 3 session 2: kernel-trace profiles of the current BERT-base, ResNet-50 and LinkNet steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3u}
mkdir -p $OUT
for m in bert-base resnet50 linknet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 8 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
  tail -1 $OUT/prof_$m.log | cut -c1-160
done
