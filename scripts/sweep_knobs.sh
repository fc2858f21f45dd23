# Interleaved whole-step A/B of engine knobs on one GPU (bench.py, 30 steps):
#   bash scripts/sweep_knobs.sh OUT_TAG "NAME ENV=VAL ..." "NAME2 ENV=VAL ..." ...
# Each round runs every config once; ROUNDS (default 2) rounds; BENCH_ARGS adds bench.py
# arguments (e.g. "--model bert-base").  One line per run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
cfgs=("$@")
mkdir -p gpurun_out/$tag
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "${cfgs[@]}"; do
    read -r -a parts <<< "$cfg"
    name=${parts[0]}
    env MLC_SWEEP=1 "${parts[@]:1}" timeout -k 10 300 python bench.py --steps 30 --warmup 8 ${BENCH_ARGS:-} \
      > gpurun_out/$tag/${name}_$r.log 2>&1 || exit 1
    echo "${name}_$r $(grep -o '"value": [0-9.]*' gpurun_out/$tag/${name}_$r.log)"
  done
done
