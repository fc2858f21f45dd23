set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q6; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests/test_transformer_gpu.py tests/test_deterministic_gpu.py tests/test_dp_gpu.py tests/test_engines_det_gpu.py tests/test_engines_gpu_vs_cpu.py tests/test_native_eval_gpu.py tests/test_graphed_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --model bert-base --steps 40 --warmup 10 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
runr() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
for r in 1 2; do
  run bert_default MLC_X=0
  runr rn_base MLC_X=0
  runr rn_deferdf MLC_WGRAD_DEFER=1 MLC_DGRAD_FIRST=1
  runr rn_df MLC_DGRAD_FIRST=1
done
python - <<'PY'
import json
for l in open('gpurun_out/q6/bench.txt'):
    tag, js = l.split(' ', 1)
    d = json.loads(js); print(tag, d['value'], d['ms_per_step'])
PY
