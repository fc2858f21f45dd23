set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for s in 1 0; do MLC_GEMM_SINGLE_STAGE=$s timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/resnet_ss$s.log 2>&1 || exit $?; echo "ss=$s $(tail -1 $OUT/resnet_ss$s.log | cut -c1-150)"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o rn -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
