#!/bin/bash
# PMC counters of the GEMM engine on conv and dense shapes (two passes, counters per pass
# within the per-block limits)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-pmc}; mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
for s in prof_convs prof_gemms; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/${s}_p1 --pmc $P1 -- python3 scripts/$s.py > $OUT/${s}_p1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/${s}_p2 --pmc $P2 -- python3 scripts/$s.py > $OUT/${s}_p2.log 2>&1 || exit $?
done
find $OUT -name "*counter_collection.csv" | head
echo "exit 0"
