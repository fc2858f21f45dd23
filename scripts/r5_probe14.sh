set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p14; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
run() { timeout -k 10 300 python -u bench.py "$@" 2>>$O/err.log | tail -1 >> $O/bench.jsonl; chk $?; }
run --model bert-base --steps 40 --warmup 10
run --steps 20 --warmup 5
run --model bert-base --steps 40 --warmup 10
run --model bert-base --steps 40 --warmup 10 --impl torch
run --model bert-base --steps 40 --warmup 10 --impl torch --precision fp32
run --steps 20 --warmup 5 --impl torch
run --steps 20 --warmup 5 --impl torch --precision fp32
run --model bert-base --steps 40 --warmup 10
run --steps 20 --warmup 5
python - <<'PY'
import json
for l in open('gpurun_out/p14/bench.jsonl'):
    d = json.loads(l); c = d['config']
    print(c['model'], c['impl'], d['dtype'], d['value'], d['ms_per_step'])
PY
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py -x -q --timeout 550 --timeout-method thread > $O/det.log 2>&1; tail -2 $O/det.log
