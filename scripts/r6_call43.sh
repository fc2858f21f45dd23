#!/bin/bash
# round-6 GPU pass 43: depthwise / generic GPU tests and smoke on the committed tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_generic_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
