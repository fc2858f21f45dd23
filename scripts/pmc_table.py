"""Pivot rocprofv3 --pmc counter CSVs into one row per dispatch (gemm kernels shortened):
python scripts/pmc_table.py A_counter_collection.csv [B_counter_collection.csv ...]"""
import csv
import re
import sys
from collections import OrderedDict

rows = OrderedDict()
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>, igemm::(\w+)', name)
        short = f'{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}/{m.group(5)}' if m else name[:40]
        if not m and 'bn_' not in name and 'Cijk' not in name:
            continue
        key = (path.split('/')[-3], int(r['Dispatch_Id']))
        d = rows.setdefault(key, {'name': short, 'us': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                                  'vgpr': r['VGPR_Count'], 'lds': r['LDS_Block_Size'], 'scr': r['Scratch_Size']})
        d[r['Counter_Name']] = float(r['Counter_Value'])
cols = sorted({c for d in rows.values() for c in d if c.isupper() or c.startswith('TCC')})
print('run/disp name us vgpr lds scratch ' + ' '.join(cols))
for (run, disp), d in rows.items():
    print(f'{run}/{disp} {d["name"]} {d["us"]:.1f} {d["vgpr"]} {d["lds"]} {d["scr"]} ' +
          ' '.join(f'{d.get(c, float("nan")):.3g}' for c in cols))
