set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q37; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_generic_gpu.py tests/test_engines_det_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; chk $rc
for m in "video:r2plus1d_18" "video:resnext3d_18"; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model $m --batch 16 --frames 8 --size 112 --classes 400 --impl native --steps 10 --warmup 3 2>>$O/err.log >> $O/gen.log; chk $?
done
cut -c1-160 $O/gen.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o v -- python3 scripts/bench_generic.py --model video:r2plus1d_18 --batch 16 --frames 8 --size 112 --classes 400 --impl native --steps 6 --warmup 3 > $O/p1.log 2>&1; chk $?
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 3 > $O/v_kernels.txt 2>&1; head -16 $O/v_kernels.txt
