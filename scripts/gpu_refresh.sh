#!/bin/bash
# Round refresh: every GPU test, smoke(), the three headline benches (ResNet-50 default
# bench.py, BERT-base, U-Net) and rocprofv3 kernel stats of each.  Stops at the first
# step that crashed / timed out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-refresh}
mkdir -p $OUT
fatal() { case $1 in 0|1) return 0;; *) echo "step $2 ended with rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -1 $OUT/smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py > $OUT/bench_resnet.log 2>&1; rc=$?; tail -1 $OUT/bench_resnet.log | cut -c1-200; fatal $rc resnet
timeout -k 10 300 python bench.py --model bert-base --steps 30 --warmup 5 > $OUT/bench_bert.log 2>&1; rc=$?; tail -1 $OUT/bench_bert.log | cut -c1-200; fatal $rc bert
timeout -k 10 300 python bench.py --model unet --steps 30 --warmup 5 > $OUT/bench_unet.log 2>&1; rc=$?; tail -1 $OUT/bench_unet.log | cut -c1-200; fatal $rc unet
for m in resnet50 bert-base unet; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o k -- python bench.py --model $m --steps 5 --warmup 3 --graph 0 > $OUT/prof_$m.log 2>&1; rc=$?
  echo "prof $m rc=$rc"; fatal $rc prof_$m
done
