"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs into per-kernel HBM bytes per launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports ½ of the bytes of a wide coalesced
(16 B/lane) streaming read -> doubled; WRITE_SIZE is exact for 16 B/lane and dword stores. Units: KB.
Usage: python scripts/pmc_summary.py FETCH.csv WRITE.csv [--workload NAME --bytes ALG_BYTES] [--json OUT]
"""
import argparse
import csv
import json
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter:
            vals[r['Kernel_Name'][:80]].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('fetch')
    p.add_argument('write')
    p.add_argument('--workload')
    p.add_argument('--bytes', type=float)
    p.add_argument('--json')
    p.add_argument('--source', default='')
    p.add_argument('--select', default='autodiffop', help='substring of the kernel names of the workload')
    p.add_argument('--git-head', default='', help='the commit the passes ran at')
    p.add_argument('--kernel-sha', default='', help="bench.py's roofline.kernel_sha16 of the measured launches")
    a = p.parse_args()
    f = per_kernel(a.fetch, 'FETCH_SIZE')
    w = per_kernel(a.write, 'WRITE_SIZE')
    out = {}
    for k in sorted(set(f) | set(w)):
        rd = 2 * f.get(k, 0.0) * 1024
        wr = w.get(k, 0.0) * 1024
        out[k] = {'read_bytes_corrected': rd, 'write_bytes': wr, 'total': rd + wr}
        print(f"{k[:60]:60s} read {rd / 1e9:8.3f} GB  write {wr / 1e9:8.3f} GB  total {(rd + wr) / 1e9:8.3f} GB")
    if a.json and a.workload:
        sel = {k: v for k, v in out.items() if a.select in k}
        entry = {'kernels': sel, 'algorithmic_bytes_per_launch': a.bytes, 'source': a.source,
                 'git_head': a.git_head, 'kernel_sha16': a.kernel_sha,
                 'note': 'FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KB->bytes, mean per launch'}
        fwd = [v['total'] for k, v in sel.items() if 'forward' in k]
        entry['bytes_per_launch'] = fwd[0] if fwd else None
        try:
            data = json.load(open(a.json))
        except (OSError, ValueError):
            data = {}
        data[a.workload] = entry
        json.dump(data, open(a.json, 'w'), indent=1)


if __name__ == '__main__':
    main()
