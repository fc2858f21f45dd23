"""Roofline table of a training step from the counter passes of scripts/pmc_roofline.sh.

    python scripts/roofline_table.py gpurun_out/pmc/rn50 --marker sgd_kernel [--steps 1] [--min-pct 1]

For every kernel family (name up to its argument list; igemm tiles shortened) in the last
``--steps`` complete steps (a step ends at the last kernel of a group of ``--marker``
optimizer kernels), per step:

* ms     - summed kernel time in the FETCH pass (counter runs serialise dispatches, so this is
           stand-alone time, no stream overlap)
* F GB   - FETCH_SIZE as reported; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
           coalesced streaming read (16 B per lane, global_load and buffer_load ... lds alike;
           /opt/skills/guides/MI355X_MICROARCH.md "HBM"), so ``rd GB`` = 2 x FETCH_SIZE is the
           byte count for the streaming kernels here (every hot kernel loads 16 B per lane)
* W GB   - WRITE_SIZE (exact for 16-B stores and f32 atomics)
* TB/s   - (rd + W) / ms, and its % of the 8 TB/s HBM3E peak (6.3 TB/s is the achievable
           copy rate quoted by the guide; scripts/bench_hbm.py measured 5.1-5.3 TB/s here)
* MFMA TF/s - SQ_VALU_MFMA_BUSY_CYCLES x 1024 FLOP per busy cycle (a 32x32x16 bf16 MFMA is
           32 busy cycles for 32,768 FLOP; a 16x16x32 one 16 cycles for 16,384), and its % of
           the 2.5 PFLOP/s dense bf16 peak
* L2 hit - TCC_HIT / (TCC_HIT + TCC_MISS)
* LDS cf - SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-array cycle)
"""
import argparse
import collections
import csv
import glob
import os
import re
import sys

HBM_PEAK = 8.0e12
MFMA_PEAK = 2.5e15


def family(name):
    m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
    if m:
        return f'igemm {m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}'
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    n = re.sub(r'^_ZN12_GLOBAL__N_1\d+', '', n)
    n = re.sub(r'^_Z\d+', '', n)
    return n.split('(')[0][:70]


def load_pass(folder):
    """{dispatch_id: [name, start, end, {counter: value}]} of one pass, in start order."""
    files = glob.glob(os.path.join(folder, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        return None
    d = collections.OrderedDict()
    for r in csv.DictReader(open(sorted(files)[-1])):
        did = int(r['Dispatch_Id'])
        e = d.setdefault(did, [r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp']), {}])
        e[3][r['Counter_Name']] = e[3].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    return sorted(d.values(), key=lambda e: e[1])


def last_steps(rows, marker, steps):
    ends = [i for i, r in enumerate(rows) if marker in r[0]]
    groups = []
    for i in ends:
        if groups and i - groups[-1][-1] <= 5:
            groups[-1].append(i)
        else:
            groups.append([i])
    bounds = [g[-1] for g in groups]
    if len(bounds) < 2:
        raise SystemExit(f'fewer than two steps found (marker {marker!r})')
    n = min(steps, len(bounds) - 1)
    return rows[bounds[-n - 1] + 1: bounds[-1] + 1], n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('--marker', default='sgd_kernel')
    ap.add_argument('--steps', type=int, default=1)
    ap.add_argument('--min-pct', type=float, default=1.0, help='list kernels above this % of step time')
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    t_step = None
    for p in sorted(glob.glob(os.path.join(a.root, 'p*'))):
        if not os.path.isdir(p):
            continue
        rows = load_pass(p)
        if not rows:
            continue
        sel, n = last_steps(rows, a.marker, a.steps)
        has_fetch = any('FETCH_SIZE' in r[3] for r in sel)
        for name, t0, t1, ctr in sel:
            f = agg[family(name)]
            for k, v in ctr.items():
                f[k] += v / n
            if has_fetch:
                f['_ms'] += (t1 - t0) / 1e6 / n
                f['_calls'] += 1.0 / n
        if has_fetch:
            t_step = sum(f['_ms'] for f in agg.values())
    if not t_step:
        raise SystemExit('no FETCH_SIZE pass found under ' + a.root)
    tot_rd = sum(2 * f.get('FETCH_SIZE', 0) * 1024 for f in agg.values())
    tot_w = sum(f.get('WRITE_SIZE', 0) * 1024 for f in agg.values())
    tot_fl = sum(f.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) * 1024 for f in agg.values())
    print(f'{a.root}: {t_step:.2f} ms/step of kernels (serialised), rd {tot_rd / 1e9:.1f} GB + wr {tot_w / 1e9:.1f} GB '
          f'per step ({(tot_rd + tot_w) / t_step / 1e9:.2f} TB/s overall), MFMA {tot_fl / 1e12:.2f} TFLOP/step '
          f'({tot_fl / t_step / 1e9:.0f} TF/s overall)')
    hdr = (f'{"ms":>7} {"%step":>5} {"n":>5} {"F GB":>6} {"rd GB":>6} {"W GB":>6} {"TB/s":>5} {"%HBM":>5} '
           f'{"MFMA TF/s":>9} {"%MFMA":>5} {"L2hit":>5} {"LDScf":>5}  kernel')
    print(hdr)
    for k, f in sorted(agg.items(), key=lambda kv: -kv[1]['_ms']):
        ms = f['_ms']
        if ms / t_step * 100 < a.min_pct:
            continue
        fetch = f.get('FETCH_SIZE', 0) * 1024
        rd, w = 2 * fetch, f.get('WRITE_SIZE', 0) * 1024
        bw = (rd + w) / (ms * 1e-3) if ms else 0
        fl = f.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) * 1024
        tf = fl / (ms * 1e-3) if ms else 0
        hit, miss = f.get('TCC_HIT_sum', f.get('TCC_HIT', 0)), f.get('TCC_MISS_sum', f.get('TCC_MISS', 0))
        l2 = f'{100 * hit / (hit + miss):5.1f}' if hit + miss else '    -'
        idx = f.get('SQ_LDS_IDX_ACTIVE', 0)
        cf = f'{f.get("SQ_LDS_BANK_CONFLICT", 0) / idx:5.2f}' if idx else '    -'
        print(f'{ms:7.3f} {100 * ms / t_step:5.1f} {f["_calls"]:5.0f} {fetch / 1e9:6.2f} {rd / 1e9:6.2f} {w / 1e9:6.2f} '
              f'{bw / 1e12:5.2f} {100 * bw / HBM_PEAK:5.1f} {tf / 1e12:9.0f} {100 * tf / MFMA_PEAK:5.1f} {l2} {cf}  {k}')
    return 0


if __name__ == '__main__':
    sys.exit(main())
