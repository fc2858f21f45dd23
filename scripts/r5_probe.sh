set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q12; mkdir -p $O
chk() { rc=$1; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: stopping"; exit $rc; fi; }
for r in 1 2; do for df in 0 1; do
  MLC_DGRAD_FIRST=$df timeout -k 10 300 python -u scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native 2>>$O/err.log | sed "s/^/df$df /" >> $O/gen.log; chk $?
done; done
for m in "resnext50_32x4d --batch 128" "efficientnet-b0 --batch 256"; do for df in 0 1; do
  MLC_DGRAD_FIRST=$df timeout -k 10 300 python -u scripts/bench_generic.py --model $m --size 224 --impl native 2>>$O/err.log | sed "s/^/df$df /" >> $O/gen.log; chk $?
done; done
cut -c1-160 $O/gen.log
