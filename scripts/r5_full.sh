# full GPU suite (one process) + the deterministic engine comparison table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/full2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
MLC_DETERMINISTIC=1 timeout -k 10 600 python -u scripts/engines_det_compare.py --noise > $O/det.jsonl 2>$O/det.err; rc2=$?
python - <<'PY'
import json
for l in open('gpurun_out/full2/det.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['kind'], 'loss %.1e' % d['loss_rel_err'], 'max %.4f med %.4f' % (d['grad_rel_max'], d['grad_rel_median']),
              'noise max %.4f med %.4f' % (d.get('noise_max', -1), d.get('noise_median', -1)))
PY
exit $rc
