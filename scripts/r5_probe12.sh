set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p12; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o gen -- python3 scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native --steps 6 --warmup 3 > $O/gen_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -20 $O/gen_prof.log; exit $rc; }
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 3 > $O/gen_kernels.txt 2>&1; head -50 $O/gen_kernels.txt
