O=gpurun_out/${RUN_TAG:-g37}
tail -n 3 $O/ktest.log; tail -n 3 $O/traj.log; cat $O/ab.jsonl $O/torch.jsonl
python -c "
import json
for l in open('$O/traj.jsonl'): d=json.loads(l); print(d['arch'], round(d['mean_rel_gap'],4), round(d['max_rel_gap'],4), [round(v,3) for v in d['native_bf16'][::4]], [round(v,3) for v in d['torch_fp32'][::4]])"
