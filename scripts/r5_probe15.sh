set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p15; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --model bert-base --steps 40 --warmup 10 2>>$O/err.log | tail -1 | sed "s/^/$tag /" >> $O/bench.txt; chk $?; }
for r in 1 2; do
  run base
  run oib MLC_OPT_IN_BWD=1
  run oib16 MLC_OPT_IN_BWD=1 MLC_BUCKET_MB=16 MLC_FIRST_BUCKET_MB=4
  run oib64 MLC_OPT_IN_BWD=1 MLC_BUCKET_MB=64
done
awk '{print $1, $4, $5}' $O/bench.txt | sed 's/,//g'
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py -x -q --timeout 550 --timeout-method thread > $O/det.log 2>&1; tail -2 $O/det.log
