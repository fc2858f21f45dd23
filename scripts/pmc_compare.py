"""Mean PMC counters per GEMM kernel (name + grid) for two runs of the same program, e.g.
the register-staged vs the LDS-DMA main loop:
python scripts/pmc_compare.py LABEL_A 'A_p*/**/*_counter_collection.csv' LABEL_B 'B_p*/...'"""
import csv
import glob
import re
import sys
from collections import defaultdict

COLS = ['SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_INSTS_LDS', 'SQ_WAIT_INST_LDS',
        'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_VMEM_RD', 'SQ_WAIT_INST_ANY', 'TCC_HIT_sum', 'TCC_MISS_sum']


def load(pattern):
    agg = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(path)):
            m = re.search(r'gemm_kernel<(\d+), (\d+), igemm::(\w+)<\d+>, igemm::(\w+)<\d+>', r['Kernel_Name'])
            pf = re.search(r', (\d)>\(', r['Kernel_Name'])
            if not m or not pf:
                continue
            key = (f'{m.group(1)}x{m.group(2)} {m.group(3)}/{m.group(4)}', int(r['Grid_Size']))
            agg[key]['PF'].append(float(pf.group(1)))
            agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
            if 'Start_Timestamp' in r:
                agg[key]['us'].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    return agg


def mean(v):
    return sum(v) / len(v) if v else float('nan')


def main():
    runs = [(sys.argv[i], load(sys.argv[i + 1])) for i in range(1, len(sys.argv), 2)]
    keys = sorted(set(k for _, a in runs for k in a))
    print(f'{"kernel":36s} {"grid":>8s} {"run":>6s} {"PF":>3s} ' + ' '.join(f'{c[3:18]:>15s}' for c in COLS))
    for k in keys:
        for label, a in runs:
            if k not in a:
                continue
            d = a[k]
            print(f'{k[0]:36s} {k[1]:8d} {label:>6s} {mean(d["PF"]):3.0f} ' +
                  ' '.join(f'{mean(d[c]):15.3e}' for c in COLS))


if __name__ == '__main__':
    main()
