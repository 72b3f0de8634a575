"""Where the IMU branch's kernels land in the bench step's timeline (rocprofv3 --kernel-trace csv of a short bench):
per IMU kernel of the last traced step, its start / end relative to the step's first kernel, and every other kernel
that overlapped it with that kernel's duration against the median of its name (the slowdown it took).
    python tools/debug/imu_timeline.py TRACE_DIR"""
import collections
import csv
import glob
import statistics
import sys


def main():
    rows = []
    for fn in glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(fn)):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    dur = collections.defaultdict(list)
    for s, e, n in rows:
        dur[n].append(e - s)
    med = {n: statistics.median(v) for n, v in dur.items()}
    # steps delimited by the AdamW kernel (one per step)
    ad = [i for i, (s, e, n) in enumerate(rows) if 'mt_adamw' in n]
    if len(ad) < 2:
        print('need >= 2 steps'); return
    lo, hi = ad[-2] + 1, ad[-1] + 1
    step = rows[lo:hi]
    t0 = step[0][0]
    print(f'step: {len(step)} kernels, {(step[-1][1] - t0) / 1e3:.1f} us')
    for s, e, n in step:
        if 'imu' not in n.lower():
            continue
        ov = [(s2, e2, n2) for s2, e2, n2 in step if 'imu' not in n2.lower() and s2 < e and e2 > s]
        print(f'IMU {n[:60]:60s} {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  ({(e - s) / 1e3:.1f} us, '
              f'median {med[n] / 1e3:.1f})')
        for s2, e2, n2 in ov:
            print(f'      || {n2[:70]:70s} {(e2 - s2) / 1e3:8.1f} us (median {med[n2] / 1e3:8.1f})')


if __name__ == '__main__':
    main()
