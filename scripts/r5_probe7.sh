set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p7; mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step failed hard rc=$rc: stopping"; exit $rc; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn50c -- python3 bench.py --steps 6 --warmup 3 --comm rccl1 > $O/rn50c_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -20 $O/rn50c_prof.log; exit $rc; }
python scripts/overlap_report.py $O/prof --marker sgd_kernel --steps 3 > $O/rn50_overlap.txt 2>&1; tail -25 $O/rn50_overlap.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profb -o bertc -- python3 bench.py --model bert-base --steps 6 --warmup 4 --comm rccl1 > $O/bertc_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bertc_prof.log; exit $rc; }
python scripts/overlap_report.py $O/profb --marker adam --steps 3 > $O/bert_overlap.txt 2>&1; tail -30 $O/bert_overlap.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --comm rccl1 > $O/rn50c.json 2>$O/rn50c.err; chk $?; tail -1 $O/rn50c.json
timeout -k 10 900 python -u scripts/graph_eager_variants.py > $O/variants.log 2>&1; chk $?; grep -v amdgpu.ids $O/variants.log | tail -12
timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py -k "resnext3d or r2plus1d" -x -v --timeout 240 --timeout-method thread > $O/video.log 2>&1; chk $?; grep -E "PASS|FAIL|Error" $O/video.log | tail -8
timeout -k 10 700 python -u -m pytest tests/test_examples_gpu.py -k throughput -x -v -s --timeout 650 --timeout-method thread > $O/dagfps.log 2>&1; rc=$?
grep -E "DAG train|passed|failed|Error" $O/dagfps.log | tail -8
exit $rc
