#!/bin/bash
# round-6 GPU pass 41 (tree as committed, rebuilt .so): full GPU suite, smoke, ResNet-50 headline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_full.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_full.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/b.json 2>> $O/bench.err || exit $?
tail -1 $O/b.json
