#!/bin/bash
# round-6 GPU pass 21: one-launch zeroing / no loss copy in the ResNet-50 step - tests, bench,
# dispatch count
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_graphed_gpu.py tests/test_dp_gpu.py tests/test_dp_bench_gpu.py tests/test_examples_gpu.py tests/test_stream_isolation_gpu.py > $O/pytest.log 2>&1 || exit $?
: > $O/bench.jsonl
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  tail -1 $O/b.json >> $O/bench.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50 -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit $?
tail -1 $O/pytest.log; python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['value'], d['ms_per_step'])"
