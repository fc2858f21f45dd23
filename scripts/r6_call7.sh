#!/bin/bash
# round-6 GPU pass 7 (retry): the suspicious test sequence with HIP error logging, the full GPU
# suite, the headline bench, the ResNet-50 steady-state kernel list, smoke, then graph /
# NULL-stream with MIOpen disabled
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g
mkdir -p $O
AMD_LOG_LEVEL=1 timeout -k 10 600 python -u -m pytest tests/test_comm_watchdog_gpu.py tests/test_gtransformer_gpu.py tests/test_kernels_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_seq.log 2>&1 || { tail -60 $O/pytest_seq.log; exit 1; }
tail -2 $O/pytest_seq.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/rn50.json 2> $O/rn50.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/rn50b.json 2> $O/rn50b.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50 -- python bench.py --steps 8 --warmup 5 > $O/prof_rn50.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/rn50.json $O/rn50b.json $O/smoke.log
for mode in nomiopen nomiopen_eval null; do
  timeout -k 10 400 python -u scripts/graph_null_stream_bisect.py effnet $mode >> $O/graph_bisect.jsonl 2>> $O/graph_bisect.err || exit $?
done
cut -c1-230 $O/graph_bisect.jsonl
