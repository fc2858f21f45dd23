# round-5 probe 1: stream-isolation tests, steady-state ResNet-50 / BERT kernel lists
# with the library selection off, benches with it off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_stream_isolation_gpu.py -x -v --timeout 240 --timeout-method thread > $O/iso.log 2>&1; rc=$?
tail -5 $O/iso.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
export MLC_BLASLT=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50 -- python3 bench.py --steps 6 --warmup 3 > $O/rn50_prof.log 2>&1 || exit $?
python scripts/steady_kernels.py $O/prof --marker sgd_kernel --steps 4 > $O/rn50_kernels.txt 2>&1
head -50 $O/rn50_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profb -o bert -- python3 bench.py --model bert-base --steps 6 --warmup 4 > $O/bert_prof.log 2>&1 || exit $?
python scripts/steady_kernels.py $O/profb --marker adam --steps 4 > $O/bert_kernels.txt 2>&1
head -50 $O/bert_kernels.txt
