set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p5; mkdir -p $O
for args in "900 600 30 null" "900 600 30 created" "200 3000 30 null" "3000 200 30 null"; do
  timeout -k 10 200 python -u scripts/graph_kernarg_probe.py $args >> $O/kernarg.log 2>&1 || exit $?
done
grep -v amdgpu.ids $O/kernarg.log
