set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q22; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 300 python -u scripts/bench_expand_1x1.py > $O/expand.jsonl 2>$O/err.log; chk $?; cut -c1-200 $O/expand.jsonl
runr() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
for r in 1 2; do
  runr base MLC_X=0
  runr sskt2 MLC_SINGLE_STAGE_KT=2
  runr sskt4 MLC_SINGLE_STAGE_KT=4
done
python - <<'PY'
import json
for l in open('gpurun_out/q22/bench.txt'):
    tag, js = l.split(' ', 1)
    d = json.loads(js); print(tag, d['value'], d['ms_per_step'])
PY
