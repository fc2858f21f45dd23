"""Summarise a rocprofv3 kernel_stats.csv per training step: python scripts/prof_summary.py CSV STEPS"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'total {tot / 1e6 / steps:.3f} ms/step over {steps:g} steps')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:6.1f}x  {r['Name'][:120]}")
