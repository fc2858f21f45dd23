"""Achieved HBM bandwidth per kernel family from scripts/gpu_hbm.sh output.

usage: python scripts/hbm_table.py gpurun_out/hbm resnet50 [steps]
Joins the FETCH_SIZE and WRITE_SIZE passes per dispatch (both runs launch the same kernels in
the same order), sums bytes and kernel time per family (name up to the argument list), and
prints per-step ms, GB moved and TB/s.  Counter runs serialise the kernels, so these are
stand-alone rates (no stream overlap)."""
import collections
import csv
import glob
import os
import sys


def load(folder):
    pmc = glob.glob(os.path.join(folder, '**', '*counter_collection.csv'), recursive=True)
    rows = list(csv.DictReader(open(pmc[0])))
    vals = collections.OrderedDict()
    for r in rows:
        vals[int(r['Dispatch_Id'])] = (r['Kernel_Name'], float(r['Counter_Value']))
    tr = glob.glob(os.path.join(folder, '**', '*kernel_trace.csv'), recursive=True)
    dur = {int(r['Dispatch_Id']): (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
           for r in csv.DictReader(open(tr[0]))}
    return vals, dur


def family(name):
    n = name.replace('(anonymous namespace)::', '').split('(')[0]
    for a, b in (('void ', ''), ('igemm::', ''), ('_ZN12_GLOBAL__N_1', '')):
        n = n.replace(a, b)
    return n[:100]


def main():
    root, model = sys.argv[1], sys.argv[2]
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
    fetch, dur = load(os.path.join(root, f'{model}_FETCH_SIZE'))
    write, _ = load(os.path.join(root, f'{model}_WRITE_SIZE'))
    wl = list(write.values())
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for i, (did, (name, fkb)) in enumerate(fetch.items()):
        wkb = wl[i][1] if i < len(wl) and wl[i][0] == name else 0.0
        a = agg[family(name)]
        a[0] += (fkb + wkb) * 1024          # FETCH_SIZE / WRITE_SIZE are in KB
        a[1] += dur.get(did, 0.0)
        a[2] += 1
    tot_b = sum(a[0] for a in agg.values())
    tot_t = sum(a[1] for a in agg.values())
    print(f'{model}: {tot_t / steps * 1e3:.2f} ms/step of kernels (serialised), {tot_b / steps / 1e9:.1f} GB/step, '
          f'{tot_b / tot_t / 1e12:.2f} TB/s overall')
    print(f'{"ms/step":>8} {"GB/step":>8} {"TB/s":>6} {"n/step":>6}  kernel')
    for k, (b, t, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f'{t / steps * 1e3:8.3f} {b / steps / 1e9:8.2f} {b / max(t, 1e-12) / 1e12:6.2f} {n / steps:6.1f}  {k}')


if __name__ == '__main__':
    main()
