set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p16; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py tests/test_stream_isolation_gpu.py tests/test_engines_det_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gen_tests.log 2>&1; rc=$?; tail -2 $O/gen_tests.log; chk $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native > $O/gen.log 2>&1; chk $?
timeout -k 10 300 python -u scripts/bench_generic.py --model resnext50_32x4d --batch 128 --size 224 --impl native >> $O/gen.log 2>&1; chk $?
timeout -k 10 300 python -u scripts/bench_generic.py --model efficientnet-b0 --batch 256 --size 224 --impl native >> $O/gen.log 2>&1; chk $?
grep img_per_s $O/gen.log
