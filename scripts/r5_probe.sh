set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q38; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
for impl in native torch; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model densenet121 --batch 64 --size 224 --impl $impl --steps 10 --warmup 3 2>>$O/err.log >> $O/gen.log; chk $?
  timeout -k 10 300 python -u scripts/bench_generic.py --model inceptionv3 --batch 80 --size 299 --impl $impl --steps 10 --warmup 3 2>>$O/err.log >> $O/gen.log; chk $?
done
cut -c1-160 $O/gen.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o d -- python3 scripts/bench_generic.py --model densenet121 --batch 64 --size 224 --impl native --steps 6 --warmup 3 > $O/p1.log 2>&1; chk $?
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 3 > $O/d_kernels.txt 2>&1; head -22 $O/d_kernels.txt
