#!/bin/bash
# GEMM iteration loop: numerics of the GEMM-backed kernels, microbench, PMC pass 1 of the
# dense shapes, BERT + ResNet bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-gi}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_seg_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm.py > $OUT/gemm.log 2>&1 || exit $?
cat $OUT/gemm.log | grep -v amdgpu.ids
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc --pmc $P1 -- python3 scripts/prof_gemms.py > $OUT/pmc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert.log 2>&1 && tail -1 $OUT/bert.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/resnet.log 2>&1 && tail -1 $OUT/resnet.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --model unet --steps 20 --warmup 5 > $OUT/unet.log 2>&1 && tail -1 $OUT/unet.log | cut -c1-160
echo "exit $?"
