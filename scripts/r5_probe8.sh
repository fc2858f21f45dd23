set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p8; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50c -- python3 bench.py --steps 6 --warmup 3 --comm rccl1 > $O/rn50c_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -20 $O/rn50c_prof.log; exit $rc; }
python scripts/overlap_report.py $O/prof --marker sgd_kernel --steps 3 > $O/rn50_overlap.txt 2>&1; tail -25 $O/rn50_overlap.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profb -o bertc -- python3 bench.py --model bert-base --steps 6 --warmup 4 --comm rccl1 > $O/bertc_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bertc_prof.log; exit $rc; }
python scripts/overlap_report.py $O/profb --marker adam --steps 3 > $O/bert_overlap.txt 2>&1; tail -40 $O/bert_overlap.txt
timeout -k 10 300 python -u scripts/graph_torch_twin.py efficientnet-b0 > $O/twin.log 2>&1; chk $?
timeout -k 10 300 python -u scripts/graph_torch_twin.py efficientnet-b0 sync >> $O/twin.log 2>&1; chk $?
timeout -k 10 300 python -u scripts/graph_torch_twin.py resnext50 >> $O/twin.log 2>&1; chk $?
grep -v amdgpu.ids $O/twin.log
