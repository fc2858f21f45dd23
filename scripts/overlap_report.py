"""Collective / compute overlap of a training step from a rocprofv3 kernel trace.

    python scripts/overlap_report.py TRACE_DIR_OR_CSV [--marker sgd_kernel] [--steps 4]

For the last ``--steps`` steps (a step ends at a group of optimizer kernels matched by
``--marker``), lists every collective kernel (RCCL / NCCL names): its start relative to
the step start and to the end of backward (the last compute kernel before the optimizer
group), its duration, and the part of it that no compute kernel overlapped (exposed).
Used with ``bench.py --comm rccl1`` (one GPU, a world-1 RCCL communicator): the
production bucketer issues its bucket all-reduces on the side stream, so their placement
inside backward is visible on a single device."""
import argparse
import csv
import glob
import os
import re
import sys

COLL = re.compile(r'(?i)(nccl|rccl|oneRankReduce)')


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, u):
    c = 0
    for x, y in u:
        lo, hi = max(a, x), min(b, y)
        if hi > lo:
            c += hi - lo
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--marker', default='sgd_kernel')
    ap.add_argument('--steps', type=int, default=4)
    a = ap.parse_args()
    path = a.path
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True),
                      key=os.path.getmtime)[-1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    groups = []
    for i in ends:
        if groups and i - groups[-1][-1] <= 5:
            groups[-1].append(i)
        else:
            groups.append([i])
    if len(groups) < 2:
        print('fewer than two steps found')
        return 1
    n = min(a.steps, len(groups) - 1)
    print(path)
    tot_coll = tot_exp = 0.0
    for g0, g1 in zip(groups[-n - 1:-1], groups[-n:]):
        sel = rows[g0[-1] + 1:g1[-1] + 1]
        t0 = int(sel[0]['Start_Timestamp'])
        t_end = int(sel[-1]['End_Timestamp'])
        opt_first = g1[0] - (g0[-1] + 1)
        comp = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in sel if not COLL.search(r['Kernel_Name'])]
        bwd_end = max(int(r['End_Timestamp']) for r in sel[:opt_first] if not COLL.search(r['Kernel_Name']))
        u = union(comp)
        coll = [r for r in sel if COLL.search(r['Kernel_Name'])]
        print(f'step: {(t_end - t0) / 1e3:.1f} us, backward ends at {(bwd_end - t0) / 1e3:.1f} us, '
              f'{len(coll)} collective kernels')
        for r in coll:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            exp = (e - s) - covered(s, e, u)
            tot_coll += (e - s) / 1e3
            tot_exp += exp / 1e3
            print(f'  start {(s - t0) / 1e3:9.1f} us ({(s - bwd_end) / 1e3:+9.1f} vs backward end)  '
                  f'{(e - s) / 1e3:7.1f} us  exposed {exp / 1e3:6.1f} us  {r["Kernel_Name"][:60]}')
    print(f'per step: collective kernel time {tot_coll / n:.1f} us, exposed {tot_exp / n:.1f} us')
    return 0


if __name__ == '__main__':
    sys.exit(main())
