# full GPU suite (one process), the deterministic engine comparison table, the flagship benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${FULL_OUT:-full}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
MLC_DETERMINISTIC=1 timeout -k 10 600 python -u scripts/engines_det_compare.py --noise > $O/det.jsonl 2>$O/det.err; rc=$?
O=$O python - <<'PY'
import json, os
for l in open(os.environ['O'] + '/det.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['kind'], 'loss %.1e' % d['loss_rel_err'], 'max %.4f med %.4f' % (d['grad_rel_max'], d['grad_rel_median']),
              'noise max %.4f med %.4f' % (d.get('noise_max', -1), d.get('noise_median', -1)))
PY
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_rn50.json 2>$O/bench.err && timeout -k 10 300 python -u bench.py --model bert-base --steps 40 --warmup 10 > $O/bench_bert.json 2>>$O/bench.err
rc=$?; cat $O/bench_rn50.json $O/bench_bert.json | cut -c1-200
exit $rc
