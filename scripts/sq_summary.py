"""Mean per dispatch of SQ/GRBM counters from rocprofv3 --pmc CSVs (one file per pass), for the kernels whose name
contains ``--select``, with the ratios DESIGN.md quotes (wait fraction, VALU-active fraction, LDS conflict share).

usage: python scripts/sq_summary.py pass1.csv pass2.csv --select stencil27_f16 [--header "# ..."]"""
import argparse
import csv
from collections import defaultdict


def collect(paths, select):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p, newline='') as f:
            for row in csv.DictReader(f):
                if select in row['Kernel_Name']:
                    acc[row['Kernel_Name']][row['Counter_Name']].append(float(row['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv', nargs='+')
    ap.add_argument('--select', required=True)
    ap.add_argument('--header', default='')
    a = ap.parse_args()
    if a.header:
        print(a.header)
    for k, c in sorted(collect(a.csv, a.select).items()):
        print(k, ' '.join(f'{n}={v:.4g}' for n, v in sorted(c.items())))
        r = []
        if 'SQ_WAIT_ANY' in c and c.get('SQ_WAVE_CYCLES'):
            r.append(f"SQ_WAIT_ANY / SQ_WAVE_CYCLES = {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        if 'SQ_WAIT_INST_ANY' in c and c.get('SQ_WAVE_CYCLES'):
            r.append(f"SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES = {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        if 'SQ_ACTIVE_INST_VALU' in c and c.get('SQ_WAVE_CYCLES'):
            r.append(f"SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES = {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}")
        if 'SQ_LDS_BANK_CONFLICT' in c and c.get('SQ_LDS_IDX_ACTIVE'):
            r.append(f"LDS bank conflicts / LDS active = {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        if 'SQ_INSTS_VALU' in c:
            r.append(f"VALU insts {c['SQ_INSTS_VALU']:.4g}")
        print(f'  {k}: ' + ', '.join(r))


if __name__ == '__main__':
    main()
