set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q3; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 500 python -u -m pytest tests/test_generic_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gen_tests.log 2>&1; chk $?; tail -2 $O/gen_tests.log
for r in 1 2; do for wt in 1 0; do
  MLC_GENERIC_WT=$wt timeout -k 10 300 python -u scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native 2>>$O/err.log | sed "s/^/wt$wt /" >> $O/gen.log; chk $?
done; done
for m in "resnext50_32x4d --batch 128" "efficientnet-b0 --batch 256"; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model $m --size 224 --impl native >> $O/gen.log 2>>$O/err.log; chk $?
done
cut -c1-160 $O/gen.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o gen -- python3 scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native --steps 6 --warmup 3 > $O/gen_prof.log 2>&1; chk $?
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 3 > $O/gen_kernels.txt 2>&1; head -30 $O/gen_kernels.txt
