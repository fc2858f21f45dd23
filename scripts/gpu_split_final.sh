#!/bin/bash
# Re-tuned split-K targets: full GPU suite, then new defaults vs the old ones (env override)
# on the three benches, then a ResNet-50 kernel summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-splitfinal}
mkdir -p $OUT
fatal() { case $1 in 0) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; fatal $rc smoke
for i in 1 2; do
  timeout -k 10 300 python bench.py > $OUT/resnet_new_$i.log 2>&1; rc=$?; fatal $rc resnet
  MLC_SPLIT_TARGET=768 MLC_SPLIT_TARGET_MAT=256 timeout -k 10 300 python bench.py > $OUT/resnet_old_$i.log 2>&1; rc=$?; fatal $rc resnet
  echo "resnet new: $(tail -1 $OUT/resnet_new_$i.log | cut -c60-100)  old: $(tail -1 $OUT/resnet_old_$i.log | cut -c60-100)"
done
for m in unet bert-base; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > $OUT/${m}_new.log 2>&1; rc=$?; fatal $rc $m
  MLC_SPLIT_TARGET=768 MLC_SPLIT_TARGET_MAT=256 timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > $OUT/${m}_old.log 2>&1; rc=$?; fatal $rc $m
  echo "$m new: $(tail -1 $OUT/${m}_new.log | cut -c60-100)  old: $(tail -1 $OUT/${m}_old.log | cut -c60-100)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_resnet50 -o k -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof_resnet50.log 2>&1; rc=$?
echo "prof rc=$rc"
