# Interleaved in-step A/B of environment configurations on one GPU box (how the round-5
# profiles/round5/*_ab*.txt tables were taken).  Run through gpurun, e.g.
#   gpurun -- 'CONFIGS="base;MLC_WGRAD_SLAB=0" ROUNDS=2 BENCH="bench.py --steps 30 --warmup 10" bash scripts/r5_probe.sh'
# Each config runs once per round, in order, so box drift hits every config alike; one line
# per run goes to gpurun_out/ab.log.
set -e
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-base}
ROUNDS=${ROUNDS:-2}
BENCH=${BENCH:-bench.py --steps 30 --warmup 10}
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in $(seq "$ROUNDS"); do
  for cfg in "${CFG[@]}"; do
    e=""; [ "$cfg" != base ] && e="$cfg"
    env $e timeout -k 10 300 python -u $BENCH > gpurun_out/ab_run.txt 2>/dev/null
    echo "$cfg $(tail -1 gpurun_out/ab_run.txt)" >> gpurun_out/ab.log
  done
done
