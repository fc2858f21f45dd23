"""Steady-state per-kernel time of a training step from a rocprofv3 kernel trace.

    python scripts/steady_kernels.py TRACE_DIR_OR_CSV [--marker sgd_kernel] [--steps 5]

Takes the last ``--steps`` complete steps of the trace (a step ends at the last kernel of
a group of optimizer kernels matched by ``--marker``), so warm-up, graph capture and any
one-off timing runs are excluded.  Prints ms per step per kernel (summed device time),
the step's wall span, and every vendor-library kernel (MIOpen, hipBLASLt / Tensile,
rocBLAS, CK): a native step must list none."""
import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict

LIB = re.compile(r'(?i)(miopen|^Cijk_|rocblas|hipblaslt|naive_conv|igemm_(fwd|bwd|wrw)_gtc|gridwise_|ck::|'
                 r'device_grouped_conv|batchnorm(fwd|bwd)|Op[1-5]dTensor|SubTensorOp|transpose_NCHW|'
                 r'kernel_batched_gemm|tensile)')


def short(name):
    m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
    if m:
        return f'igemm {m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}'
    name = re.sub(r'^void ', '', name)
    return name[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--marker', default='sgd_kernel')
    ap.add_argument('--steps', type=int, default=5)
    a = ap.parse_args()
    path = a.path
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
        if not cands:
            print('no kernel_trace.csv under', path)
            return 1
        path = sorted(cands, key=os.path.getmtime)[-1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    groups = []
    for i in ends:
        if groups and i - groups[-1][-1] <= 5:
            groups[-1].append(i)
        else:
            groups.append([i])
    bounds = [g[-1] for g in groups]
    if len(bounds) < 2:
        print(f'fewer than two steps found (marker {a.marker!r})')
        return 1
    n = min(a.steps, len(bounds) - 1)
    lo, hi = bounds[-n - 1] + 1, bounds[-1] + 1
    sel = rows[lo:hi]
    tot = defaultdict(float)
    calls = defaultdict(int)
    for r in sel:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        tot[r['Kernel_Name']] += d
        calls[r['Kernel_Name']] += 1
    span = (int(sel[-1]['End_Timestamp']) - int(sel[0]['Start_Timestamp'])) / 1e6 / n
    busy = sum(tot.values()) / n
    print(f'{path}\nlast {n} steps: wall span {span:.3f} ms/step, summed kernel time {busy:.3f} ms/step, '
          f'{len(sel) / n:.0f} dispatches/step, {len(tot)} distinct kernels')
    for k in sorted(tot, key=lambda k: -tot[k])[:45]:
        print(f'{tot[k] / n:8.3f} ms {calls[k] / n:6.1f}x  {short(k)}')
    lib = [k for k in tot if LIB.search(k)]
    print(f'library kernels: {len(lib)}')
    for k in lib:
        print(f'  LIB {tot[k] / n:8.3f} ms {calls[k] / n:6.1f}x  {k[:110]}')
    return 0


if __name__ == '__main__':
    sys.exit(main())
