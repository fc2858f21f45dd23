#!/bin/bash
# round 3 session 2: segmentation GPU tests (incl. native FPN), FPN native vs stock bench,
# kernel-trace profiles of the BERT-base, ResNet-50 and LinkNet steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3v}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_seg_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --model fpn --steps 20 --warmup 5 > $OUT/fpn_native.log 2>&1 || { echo "bench rc=$?"; tail -30 $OUT/fpn_native.log; exit 1; }
tail -1 $OUT/fpn_native.log | cut -c1-200
timeout -k 10 300 python bench.py --model fpn --impl torch --steps 20 --warmup 5 > $OUT/fpn_torch.log 2>&1 || { echo "bench torch rc=$?"; tail -30 $OUT/fpn_torch.log; exit 1; }
tail -1 $OUT/fpn_torch.log | cut -c1-200
for m in bert-base resnet50 linknet fpn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 8 --warmup 3 > $OUT/prof_$m.log 2>&1 || { echo "prof $m rc=$?"; tail -20 $OUT/prof_$m.log; exit 1; }
  tail -1 $OUT/prof_$m.log | cut -c1-120
done
