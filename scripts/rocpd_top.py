"""Top kernels of a rocprofv3 rocpd database (``*_results.db``): total ms per kernel name over
the last ``--last`` fraction of the trace (the timed steps), per step.

    python scripts/rocpd_top.py gpurun_out/prof/x_results.db --steps 5 --last 0.6
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--steps', type=int, default=5, help='timed steps inside the --last window')
    ap.add_argument('--last', type=float, default=0.5, help='fraction of dispatches (by start time) kept')
    ap.add_argument('--top', type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute('select name, start, end from kernels order by start'))
    rows = rows[int(len(rows) * (1 - a.last)):]
    span = (rows[-1][2] - rows[0][1]) / 1e6
    agg = {}
    for name, s, e in rows:
        t, n = agg.get(name, (0.0, 0))
        agg[name] = (t + (e - s) / 1e6, n + 1)
    tot = sum(t for t, _ in agg.values())
    print(f'{len(rows)} dispatches, span {span / a.steps:.3f} ms/step, summed kernel time {tot / a.steps:.3f} ms/step')
    for name, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f'{t / a.steps:9.3f} ms {n / a.steps:7.1f}x  {name[:110]}')


if __name__ == '__main__':
    main()
