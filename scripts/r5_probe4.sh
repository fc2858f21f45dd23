set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p4; mkdir -p $O
timeout -k 10 900 python -u scripts/graph_eager_variants.py > $O/variants.log 2>&1; rc=$?
grep -v amdgpu.ids $O/variants.log | tail -20
exit $rc
