set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q35; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gate_gpu.py tests/test_generic_gpu.py tests/test_engines_det_gpu.py tests/test_seg_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; chk $rc
for m in "efficientnet-b0 --batch 256" "resnext50_32x4d --batch 128" "resnet50 --batch 512"; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model $m --impl native 2>>$O/err.log >> $O/gen.log; chk $?
done
cut -c1-140 $O/gen.log
