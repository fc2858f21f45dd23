set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q16; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests/test_seg_gpu.py tests/test_engines_det_gpu.py tests/test_engines_gpu_vs_cpu.py tests/test_examples_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
runs() { tag=$1; m=$2; shift; shift; env "$@" timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
for r in 1 2; do for m in unet pspnet deeplab; do
  runs ${m}_default $m MLC_X=0
  runs ${m}_join $m MLC_WGRAD_DEFER=0
done; done
python - <<'PY'
import json
for l in open('gpurun_out/q16/bench.txt'):
    tag, js = l.split(' ', 1)
    d = json.loads(js); print(tag, d['value'], d['ms_per_step'])
PY
