set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN_TAG}; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o rn -- python bench.py --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
