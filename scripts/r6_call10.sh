#!/bin/bash
# round-6 GPU pass 10: 3D residual gradients summed in the temporal fold (tests, video
# bench + kernel trace), PSPNet anchor bisection
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_generic_gpu.py \
  -k "temporal or video or resnext3d or r2plus1d" > $O/pytest_k.log 2>&1 || exit $?
MLC_DETERMINISTIC=1 timeout -k 10 300 python -u scripts/psp_bisect.py > $O/psp_bisect.jsonl 2> $O/psp_bisect.err || exit $?
: > $O/video.jsonl
for m in r2plus1d_18 resnext3d_18 resnext3d_18; do
  timeout -k 10 300 python -u scripts/bench_generic.py --model video:$m --batch 16 --size 112 --frames 8 --classes 400 --impl native >> $O/video.jsonl 2>> $O/video.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o r3d -- python scripts/bench_generic.py --model video:resnext3d_18 --batch 16 --size 112 --frames 8 --classes 400 --impl native --steps 6 --warmup 3 > $O/prof_r3d.log 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_k.log | tail -3; cat $O/video.jsonl; python -c "
import json
for l in open('$O/psp_bisect.jsonl'):
    d=json.loads(l); print('%-10s gpu %.3g noise %.3g ratio %.2f' % (d['stage'], d['gpu_vs_cpu'], d['fp32ulp_noise'], d['ratio']))"
