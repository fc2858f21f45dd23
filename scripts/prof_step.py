"""Per-dispatch listing of the last training step in a rocprofv3 kernel trace
(step boundary = the optimizer kernel): python scripts/prof_step.py TRACE.csv [marker]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else 'sgd_kernel'
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
# the optimizer may launch >1 kernel per step: group consecutive ones
bounds = []
for i in ends:
    if not bounds or i - bounds[-1] > 5:
        bounds.append(i)
a, b = bounds[-2] + 1, bounds[-1] + 1
tot = 0
for r in rows[a:b]:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    name = r['Kernel_Name']
    m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
    short = f'gemm{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}' if m else name[:60]
    grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z']) // int(r['Workgroup_Size_X'])
    print(f'{d:9.1f} us  wg={grid:6d} vgpr={r["VGPR_Count"]:>4} {short}')
print(f'step total {tot / 1e3:.3f} ms')
