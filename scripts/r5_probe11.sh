set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p11; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
MLC_DETERMINISTIC=1 timeout -k 10 900 python -u scripts/engines_det_compare.py > $O/det.log 2>&1; chk $?
grep -v amdgpu.ids $O/det.log | cut -c1-400
timeout -k 10 300 python -u scripts/bench_generic.py --model resnet50 --batch 512 --size 224 --impl native > $O/gen_rn50.log 2>&1; chk $?
tail -1 $O/gen_rn50.log
timeout -k 10 300 python -u scripts/bench_generic.py --model resnet50 --batch 256 --size 224 --impl native >> $O/gen_rn50.log 2>&1; chk $?
tail -1 $O/gen_rn50.log
