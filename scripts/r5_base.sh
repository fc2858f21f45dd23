set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5base
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5base/rn50.json 2>gpurun_out/r5base/rn50.err &&
timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > gpurun_out/r5base/bert_auto.json 2>gpurun_out/r5base/bert_auto.err &&
MLC_BLASLT=0 timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > gpurun_out/r5base/bert_off.json 2>gpurun_out/r5base/bert_off.err
cat gpurun_out/r5base/*.json
