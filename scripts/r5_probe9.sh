set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p9; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
for mode in "" sync estream gstream; do
  timeout -k 10 300 python -u scripts/graph_torch_twin.py resnext50 $mode >> $O/twin.log 2>&1; chk $?
done
timeout -k 10 300 python -u scripts/graph_torch_twin.py cifarnet >> $O/twin.log 2>&1; chk $?
timeout -k 10 300 python -u scripts/graph_torch_twin.py resnext50 >> $O/twin.log 2>&1; chk $?
grep -v amdgpu.ids $O/twin.log
timeout -k 10 300 python -u -m pytest tests/test_stream_isolation_gpu.py -x -v --timeout 240 --timeout-method thread > $O/iso.log 2>&1; rc=$?
tail -3 $O/iso.log
exit $rc
