set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q24; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests/test_generic_gpu.py tests/test_engines_det_gpu.py tests/test_seg_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; chk $rc
for m in "unet:resnext50_32x4d --batch 16 --size 256 --classes 2" "deeplab:mobilenet --batch 16 --size 256 --classes 21" "psp:resnet34 --batch 32 --size 256 --classes 21" "fpn:resnext50_32x4d --batch 16 --size 256 --classes 2"; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model $m --impl native 2>>$O/err.log >> $O/gen.log; chk $?
done
cut -c1-150 $O/gen.log
