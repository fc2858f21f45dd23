set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_blaslt_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tx.log 2>&1; rc=$?
tail -4 $O/tx.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python -u scripts/graph_null_stream_probe.py 20 > $O/nullprobe.log 2>&1 || exit $?
grep -v amdgpu.ids $O/nullprobe.log
timeout -k 10 600 python -u scripts/graph_eager_variants.py > $O/variants.log 2>&1; rc=$?
grep -v amdgpu.ids $O/variants.log | tail -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/bert.json 2>$O/bert.err; cat $O/bert.json
