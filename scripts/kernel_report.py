"""Per-kernel time of a rocprofv3 --kernel-trace --stats run, with library kernels flagged.

    python scripts/kernel_report.py PROF_DIR NAME [STEPS]

Finds ``*NAME*kernel_stats.csv`` under PROF_DIR, prints ms per step per kernel and the
total, and lists every kernel that belongs to a vendor library (MIOpen, hipBLASLt /
Tensile, rocBLAS, composable-kernel instances MIOpen dispatches): the native engines'
steps must list none ("library kernels: 0")."""
import csv
import glob
import os
import re
import sys

LIB = re.compile(r'(?i)(miopen|^Cijk_|rocblas|hipblaslt|naive_conv|igemm_(fwd|bwd|wrw)_gtc|gridwise_|ck::|'
                 r'device_grouped_conv|batchnorm(fwd|bwd)|Op[1-5]dTensor|SubTensorOp|transpose_NCHW|'
                 r'MIOpen|kernel_batched_gemm|tensile)')


def main():
    root, name = sys.argv[1], sys.argv[2]
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    files = [f for f in glob.glob(os.path.join(root, '**', '*kernel_stats.csv'), recursive=True)
             if name in os.path.basename(f) or name in f]
    if not files:
        print(f'no kernel_stats.csv for {name} under {root}')
        return 1
    rows = list(csv.DictReader(open(sorted(files)[-1])))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print(f'{sorted(files)[-1]}\ntotal {tot / 1e6 / steps:.3f} ms/step over {steps:g} steps, {len(rows)} kernels')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:7.1f}x  {r['Name'][:110]}")
    lib = [r for r in rows if LIB.search(r['Name'])]
    print(f'library kernels: {len(lib)}')
    for r in lib:
        print(f"  LIB {float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:7.1f}x  {r['Name'][:110]}")
    return 0


if __name__ == '__main__':
    sys.exit(main())
