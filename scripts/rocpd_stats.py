"""Per-kernel statistics from a rocprofv3 SQLite trace (``rocprofv3 --kernel-trace -d DIR
-o run``, ROCm 7 writes ``DIR/.../run_results.db``): name, calls, total and mean duration,
VGPR count, per step when ``--steps`` is given (the profiled bench's timed + warm-up steps
are all in the trace; the per-step column divides by --steps).

    python scripts/rocpd_stats.py gpurun_out/r3c/prof_bert-base --steps 11 [--top 40] [--csv out.csv]
"""
import argparse
import csv
import glob
import os
import re
import sqlite3


def short(name: str) -> str:
    n = re.sub(r'\(anonymous namespace\)::|_GLOBAL__N_1|igemm::', '', name)
    m = re.match(r'void gemm_kernel<(\d+), (\d+), (\w+)<\d+>, (\w+)<\d+>, (\w+)(?:<[^>]*>)?, (\d)>', n)
    if m:
        return f'gemm{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)} pf{m.group(6)}'
    return n.split('(')[0][:90]


def load(path):
    dbs = glob.glob(os.path.join(path, '**', '*.db'), recursive=True) if os.path.isdir(path) else [path]
    rows = []
    for d in dbs:
        con = sqlite3.connect(d)
        rows += con.execute('select name, duration, vgpr_count, accum_vgpr_count, grid_x, workgroup_x, '
                            'queue_id, start, end from kernels').fetchall()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--steps', type=float, default=1.0)
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--csv', default='')
    a = ap.parse_args()
    rows = load(a.path)
    agg = {}
    for name, dur, vg, ag, gx, wx, q, s, e in rows:
        k = agg.setdefault(name, [0, 0, vg + ag, gx // max(wx, 1)])
        k[0] += 1
        k[1] += dur
    tot = sum(v[1] for v in agg.values())
    span = (max(r[8] for r in rows) - min(r[7] for r in rows)) if rows else 0
    print(f'kernels {len(rows)}  summed {tot / 1e6:.3f} ms  span {span / 1e6:.3f} ms  '
          f'per step: summed {tot / 1e6 / a.steps:.3f} ms')
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f'{"us/step":>9} {"calls/st":>8} {"avg us":>8} {"vgpr":>5} {"blocks":>7}  kernel')
    for name, (c, t, vg, blk) in out[:a.top]:
        print(f'{t / 1e3 / a.steps:9.1f} {c / a.steps:8.1f} {t / c / 1e3:8.1f} {vg:5d} {blk:7d}  {short(name)}')
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'calls', 'total_ns', 'avg_ns', 'us_per_step', 'vgpr', 'blocks'])
            for name, (c, t, vg, blk) in out:
                w.writerow([name, c, t, t // c, round(t / 1e3 / a.steps, 1), vg, blk])


if __name__ == '__main__':
    main()
