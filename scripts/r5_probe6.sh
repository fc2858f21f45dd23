set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p6; mkdir -p $O
MLC_WORK_STREAM=0 timeout -k 10 300 python -u scripts/graph_eager_bisect.py > $O/bisect.log 2>&1; rc=$?
grep -v amdgpu.ids $O/bisect.log | tail -30
exit $rc
