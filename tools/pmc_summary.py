"""Summarise a rocprofv3 --pmc CSV (counter_collection.csv): per kernel, the mean of each counter per dispatch.
python tools/pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    files = glob.glob(f'{path}/**/*counter_collection.csv', recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = r['Kernel_Name']
                if filt not in k:
                    continue
                acc[k][r['Counter_Name']] += float(r['Counter_Value'])
                disp[k].add(r['Dispatch_Id'])
    for k, cs in sorted(acc.items(), key=lambda kv: kv[0]):
        n = len(disp[k])
        print(k[:90], f'dispatches={n}')
        for c, v in sorted(cs.items()):
            print(f'    {c:32s} {v / n:16.4g}')


if __name__ == '__main__':
    main()
