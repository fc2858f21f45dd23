set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p2; mkdir -p $O
timeout -k 10 120 python -u scripts/graph_null_stream_probe.py 20 > $O/nullprobe.log 2>&1; rc=$?
cat $O/nullprobe.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/graph_eager_variants.py > $O/variants.log 2>&1; rc=$?
grep -v amdgpu.ids $O/variants.log | tail -20
exit $rc
