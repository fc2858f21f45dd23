set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q10; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dp_bench_gpu.py -x -v --timeout 280 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -30 $O/tests.log; exit $rc
