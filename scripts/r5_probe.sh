set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q11; mkdir -p $O
CONV_ONLY=1 CONV_BATCH=512 timeout -k 10 300 python -u scripts/bench_gemm256.py > $O/conv512.log 2>&1; rc=$?; cat $O/conv512.log | grep conv; exit $rc
