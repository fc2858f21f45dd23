set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q9; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --model bert-base --steps 40 --warmup 10 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
for r in 1 2; do
  run default MLC_X=0
  run wsplit192 MLC_SPLIT_TARGET_DENSE=192
  run wsplit320 MLC_SPLIT_TARGET_DENSE=320
  run wsplit256 MLC_SPLIT_TARGET_DENSE=256
done
python - <<'PY'
import json
for l in open('gpurun_out/q9/bench.txt'):
    tag, js = l.split(' ', 1)
    d = json.loads(js); print(tag, d['value'], d['ms_per_step'])
PY
