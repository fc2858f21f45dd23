#!/bin/bash
# The one GPU launcher (replaces the per-experiment gpu_*.sh scripts of rounds 1-3).
# Run on the GPU box through gpurun, e.g.
#   gpurun --timeout 900 -- 'bash scripts/gpu.sh tests tests/test_generic_gpu.py && bash scripts/gpu.sh bench'
#
#   tests [PATHS...]        pytest -m gpu (one process, per-test timeout) -> $OUT/pytest.log
#   bench [ARGS...]         python bench.py ARGS -> $OUT/bench.json (the driver's headline line)
#   prof NAME -- CMD...     rocprofv3 --kernel-trace --stats of CMD -> $OUT/prof/NAME*, summary
#                           (scripts/kernel_report.py: library kernels flagged) -> $OUT/NAME_kernels.txt
#   pmc NAME COUNTERS -- CMD...  one counter pass (rocprofv3 --pmc; <= 8 SQ / 4 TCC ...)
#   run NAME -- CMD...      any command, output -> $OUT/NAME.log
# Every GPU step runs under its own `timeout -k 10` (STEP_TIMEOUT, default 600 s); the first
# failing step ends the script with its exit status (chain modes with &&, never retry).
# OUT = gpurun_out/${RUN_TAG:-run}.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-run}
mkdir -p "$OUT"
T=${STEP_TIMEOUT:-600}
mode=$1; shift

split_cmd() {   # NAME -- CMD...  ->  NAME, CMD
  NAME=$1; shift
  [ "$1" == "--" ] && shift
  CMD=("$@")
}

case "$mode" in
  tests)
    timeout -k 10 "$T" python -u -m pytest "${@:-tests}" -m gpu -x -v --timeout 240 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1; rc=$?
    tail -5 "$OUT/pytest.log"; exit $rc ;;
  bench)
    timeout -k 10 "$T" python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
    tail -2 "$OUT/bench.json"; tail -3 "$OUT/bench.err"; exit $rc ;;
  prof)
    split_cmd "$@"
    timeout -k 10 "$T" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o "$NAME" -- "${CMD[@]}" \
      > "$OUT/${NAME}_prof.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -20 "$OUT/${NAME}_prof.log"; exit $rc; }
    python scripts/kernel_report.py "$OUT/prof" "$NAME" "${STEPS:-1}" > "$OUT/${NAME}_kernels.txt" 2>&1
    head -40 "$OUT/${NAME}_kernels.txt"; exit 0 ;;
  pmc)
    NAME=$1; COUNTERS=$2; shift 2; [ "$1" == "--" ] && shift
    timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --output-format csv -d "$OUT/pmc" -o "$NAME" -- "$@" \
      > "$OUT/${NAME}_pmc.log" 2>&1; rc=$?
    tail -5 "$OUT/${NAME}_pmc.log"; exit $rc ;;
  run)
    split_cmd "$@"
    timeout -k 10 "$T" "${CMD[@]}" > "$OUT/$NAME.log" 2>&1; rc=$?
    tail -30 "$OUT/$NAME.log"; exit $rc ;;
  *)
    echo "usage: gpu.sh tests|bench|prof|pmc|run ..." >&2; exit 2 ;;
esac
