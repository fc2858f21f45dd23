"""Idle time inside one training step of a rocprofv3 kernel trace: the step's wall span
(first kernel start -> last kernel end, steps delimited by the optimizer kernel), the union
of busy intervals over all streams, and the largest windows with no kernel running.

    python scripts/step_gaps.py TRACE_kernel_trace.csv [marker=sgd_kernel] [top=15]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
    if m:
        return f'gemm{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}'
    m = re.search(r'N12_GLOBAL__N_1\d+(\w+?)_kernel', name)
    return (m.group(1) + '_kernel') if m else name[:50]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker = sys.argv[2] if len(sys.argv) > 2 else 'sgd_kernel'
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    bounds = []
    for i in ends:
        if not bounds or i - bounds[-1] > 5:
            bounds.append(i)
    a, b = bounds[-2] + 1, bounds[-1] + 1
    step = rows[a:b]
    iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in step]
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    busy, gaps = 0, []
    cur_s, cur_e, cur_n = iv[0]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_n, n))
            cur_s, cur_e, cur_n = s, e, n
        elif e > cur_e:
            cur_e, cur_n = e, n
    busy += cur_e - cur_s
    span = t1 - t0
    print(f'kernels {len(iv)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  '
          f'idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps '
          f'(mean {(span - busy) / max(1, len(gaps)) / 1e3:.2f} us)')
    hist = {}
    for g, _, _ in gaps:
        k = '<2us' if g < 2e3 else '2-5us' if g < 5e3 else '5-20us' if g < 2e4 else '>=20us'
        hist[k] = hist.get(k, 0) + g
    print('idle by gap size: ' + ', '.join(f'{k} {v / 1e3:.0f} us' for k, v in hist.items()))
    for g, p, n in sorted(gaps, reverse=True)[:top]:
        print(f'{g / 1e3:8.1f} us  after {short(p):48s} before {short(n)}')


if __name__ == '__main__':
    main()
