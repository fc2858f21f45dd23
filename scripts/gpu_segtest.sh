set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/seg2
timeout -k 10 300 python -u -m pytest tests/test_seg_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/seg2/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/seg2/pytest.log; exit $rc
