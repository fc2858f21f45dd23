#!/bin/bash
# round-6 first GPU pass: headline bench, RCCL failure handling, counter passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/rn50.json 2> $O/rn50.err &&
timeout -k 10 300 python -u -m pytest tests/test_comm_watchdog_gpu.py tests/test_native_gpu.py -k "watchdog or never_joins or world1 or rccl or data_parallel" -x -v --timeout 120 --timeout-method thread > $O/pytest_comm.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --comm rccl1 > $O/rn50_rccl1.json 2> $O/rn50_rccl1.err &&
bash scripts/pmc_roofline.sh rn50 -- python bench.py --graph 0 --steps 2 --warmup 1 &&
bash scripts/pmc_roofline.sh bert -- python bench.py --model bert-base --graph 0 --steps 2 --warmup 1
rc=$?
cat $O/*.json; tail -3 $O/pytest_comm.log
exit $rc
