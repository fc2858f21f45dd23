#!/bin/bash
# Hardware-counter capture of a training step for the roofline table
# (scripts/roofline_table.py).  Run on the GPU box through gpurun:
#
#   gpurun --timeout 1200 -- 'bash scripts/pmc_roofline.sh rn50 -- python bench.py --graph 0 --steps 2 --warmup 1'
#
# One rocprofv3 run per counter pass (gfx950 slots: 8 SQ, 4 TCC, 2 GRBM; FETCH_SIZE takes
# 3 TCC and WRITE_SIZE 2, so they get a pass each), the program directly after `--`.
# Passes whose counters this rocprofv3 does not list are skipped (rocprofv3 -L is saved).
# Each pass runs under its own `timeout -s KILL`; the first failing pass ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NAME=$1; shift
[ "$1" == "--" ] && shift
OUT=gpurun_out/pmc/$NAME
mkdir -p "$OUT"
T=${PASS_TIMEOUT:-240}
[ -s gpurun_out/pmc/counters.txt ] || timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1

PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"
  "TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  keep=""
  for c in $P; do
    base=${c%_sum}
    if grep -q -w "$base" gpurun_out/pmc/counters.txt; then keep="$keep $c"; else echo "skip counter $c (not listed)"; fi
  done
  [ -z "$keep" ] && continue
  echo "[pass $i] $keep"
  timeout -s KILL "$T" rocprofv3 --pmc $keep --output-format csv -d "$OUT/p$i" -o run -- "$@" \
    > "$OUT/p$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
echo "pmc passes done: $OUT"
