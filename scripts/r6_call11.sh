#!/bin/bash
# round-6 GPU pass 11: native adaptive pool (PSPNet pyramid) - kernel tests, PSPNet
# stage bisection and the deterministic anchor for PSPNet
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_seg_gpu.py \
  -k "adaptive or temporal or psp" > $O/pytest_k.log 2>&1 || exit $?
MLC_DETERMINISTIC=1 timeout -k 10 300 python -u scripts/psp_bisect.py > $O/psp_bisect.jsonl 2> $O/psp_bisect.err || exit $?
MLC_DETERMINISTIC=1 timeout -k 10 600 python -u scripts/engines_det_compare.py --noise pspnet deeplab > $O/engines_det.jsonl 2> $O/engines_det.err || exit $?
grep -E "passed|failed" $O/pytest_k.log | tail -3; python -c "
import json
for l in open('$O/psp_bisect.jsonl'):
    d=json.loads(l); print('%-10s gpu %.3g noise %.3g' % (d['stage'], d['gpu_vs_cpu'], d['fp32ulp_noise']))
for l in open('$O/engines_det.jsonl'):
    d = json.loads(l)
    print(d['kind'], 'loss %.2e/%.2e gpu med %.3g max %.3g | noise med %.3g max %.3g | ratio med %.2f slotmax %.2f' % (
        d['loss_rel_err'], d['noise_loss_rel'], d['grad_rel_median'], d['grad_rel_max'], d['noise_median'], d['noise_max'], d['ratio_median'], d['ratio_slot_max']))"
