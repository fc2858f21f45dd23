set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p10; mkdir -p $O
timeout -k 10 300 python -u scripts/bench_g256_dense.py 4096 > $O/g256_bert.log 2>&1; rc=$?
grep -v amdgpu.ids $O/g256_bert.log
exit $rc
