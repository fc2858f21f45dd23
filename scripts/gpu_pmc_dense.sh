#!/bin/bash
# PMC passes over the dense GEMM shapes of scripts/prof_dense.py (native tiles vs hipBLASLt)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-pmcd}; mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
P3="SQ_INSTS_VMEM_WR SQ_WAIT_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$i --pmc $P -- python3 scripts/prof_dense.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 scripts/pmc_table.py $(find $OUT -name "*counter_collection.csv" | sort) > $OUT/table.txt 2>&1
cat $OUT/table.txt
