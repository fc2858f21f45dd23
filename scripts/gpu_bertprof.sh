set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3b; mkdir -p $OUT
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > $OUT/bert_native.log 2>&1 && tail -1 $OUT/bert_native.log &&
timeout -k 10 300 python bench.py --model bert-base --impl torch --steps 20 --warmup 5 > $OUT/bert_torch.log 2>&1 && tail -1 $OUT/bert_torch.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bert -- python bench.py --model bert-base --steps 5 --warmup 3 --graph 0 > $OUT/prof.log 2>&1
echo "exit $?"
