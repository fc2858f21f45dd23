"""Per-queue view of one captured training step from a rocprofv3 kernel trace: busy time
per hardware queue, time with 0 / 1 / 2+ kernels running, and the top kernels per queue.

    python scripts/queue_busy.py TRACE_kernel_trace.csv [marker=sgd_kernel]
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
    if m:
        return f'gemm{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}'
    m = re.search(r'N12_GLOBAL__N_1\d+(\w+?)_kernel', name) or re.search(r'(\w+?)_kernel', name)
    return (m.group(1) + '_kernel') if m else name[:50]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker = sys.argv[2] if len(sys.argv) > 2 else 'sgd_kernel'
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    bounds = []
    for i in ends:
        if not bounds or i - bounds[-1] > 5:
            bounds.append(i)
    a, b = bounds[-2] + 1, bounds[-1] + 1
    while b < len(rows) and marker in rows[b]['Kernel_Name']:
        b += 1
    step = rows[a:b]
    t0 = min(int(r['Start_Timestamp']) for r in step)
    t1 = max(int(r['End_Timestamp']) for r in step)
    print(f'step span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels')
    per_q = collections.defaultdict(list)
    for r in step:
        per_q[r['Queue_Id']].append(r)
    for q, rs in sorted(per_q.items()):
        busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rs)
        tops = collections.Counter()
        for r in rs:
            tops[short(r['Kernel_Name'])] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        print(f'queue {q}: {len(rs)} kernels, busy {busy / 1e3:.1f} us')
        for k, v in tops.most_common(8):
            print(f'    {v / 1e3:9.1f} us  {k}')
    ev = []
    for r in step:
        ev.append((int(r['Start_Timestamp']), 1))
        ev.append((int(r['End_Timestamp']), -1))
    ev.sort()
    conc = collections.Counter()
    cur, last = 0, t0
    for t, d in ev:
        conc[min(cur, 2)] += t - last
        cur += d
        last = t
    print('time with 0 / 1 / 2+ kernels running: ' + ' / '.join(f'{conc[i] / 1e3:.1f} us' for i in range(3)))


if __name__ == '__main__':
    main()
