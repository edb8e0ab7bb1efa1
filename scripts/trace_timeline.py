"""Timeline of the last dispatches of a rocprofv3 kernel trace (``*_kernel_trace.csv``): start offset, duration,
idle gap since the previous dispatch ended, queue / stream, short kernel name.

python scripts/trace_timeline.py TRACE.csv [--last N] [--skip-torch]"""
import argparse
import csv


def main():
    p = argparse.ArgumentParser()
    p.add_argument('trace')
    p.add_argument('--last', type=int, default=60)
    p.add_argument('--width', type=int, default=48)
    a = p.parse_args()
    with open(a.trace) as f:
        rows = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r['Queue_Id'], r['Stream_Id'])
                for r in csv.DictReader(f)]
    rows.sort()
    rows = rows[-a.last:]
    t0 = rows[0][0]
    busy_end = t0
    busy = 0
    for s, e, name, q, st in rows:
        gap = max(0, s - busy_end)
        # union of busy intervals (concurrent kernels overlap)
        busy += max(0, e - max(s, busy_end))
        busy_end = max(busy_end, e)
        short = name.split('(')[0].replace('void ', '')[:a.width]
        print(f'{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap / 1e3:7.1f}  q{q} s{st}  {short}')
    span = busy_end - t0
    print(f'span {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us ({busy / span:.1%})')


if __name__ == '__main__':
    main()
