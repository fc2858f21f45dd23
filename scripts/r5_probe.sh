set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q30; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gate_gpu.py tests/test_generic_gpu.py tests/test_engines_det_gpu.py -x -q --timeout 600 --timeout-method thread -k "efficient or se_ or gate or resnext or chscale" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; chk $rc
for m in "efficientnet-b0 --batch 256" "se_resnext50_32x4d --batch 64"; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model $m --impl native 2>>$O/err.log >> $O/gen.log; chk $?
done
cut -c1-150 $O/gen.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o eff -- python3 scripts/bench_generic.py --model efficientnet-b0 --batch 256 --size 224 --impl native --steps 6 --warmup 3 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 3 > $O/eff_kernels.txt 2>&1; head -12 $O/eff_kernels.txt
