#!/bin/bash
# PMC counters of the GEMMs on the LDS-DMA vs the register-staged main loop (two counter
# passes per mode, within the per-block limits)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-pmcdma}; mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
for v in 0 1; do
  MLC_GEMM_DMA=$v timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/dma${v}_p1 --pmc $P1 -- python3 scripts/prof_dma.py > $OUT/dma${v}_p1.log 2>&1 || exit $?
  MLC_GEMM_DMA=$v timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/dma${v}_p2 --pmc $P2 -- python3 scripts/prof_dma.py > $OUT/dma${v}_p2.log 2>&1 || exit $?
done
find $OUT -name "*counter_collection.csv"
echo "exit 0"
