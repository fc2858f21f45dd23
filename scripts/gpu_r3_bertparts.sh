#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG:-r3e}
mkdir -p $OUT
timeout -k 10 300 python scripts/bench_bert_parts.py > $OUT/parts.log 2>&1 || { echo "parts rc=$?"; tail -20 $OUT/parts.log; exit 1; }
tail -1 $OUT/parts.log
MLC_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_serial -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > $OUT/prof_serial.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/prof_serial.log; exit 1; }
grep -o '"value": [0-9.]*' $OUT/prof_serial.log
