"""Per-kernel PMC counters from rocprofv3 --pmc passes (one directory per pass), averaged per dispatch.

    python tools/debug/pmc_table.py FILTER DIR [DIR ...]

Prints, for every kernel whose name contains FILTER, each counter per dispatch and — when GRBM_GUI_ACTIVE was
collected in the same pass — per kernel cycle (GRBM_GUI_ACTIVE / 8 XCDs) and per SIMD (÷ 1024 SIMDs).  SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles summed over waves (MI355X_MICROARCH.md constants table);
SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs."""
import collections
import csv
import glob
import sys


def main():
    filt, dirs = sys.argv[1], sys.argv[2:]
    tab = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for fn in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
            with open(fn) as f:
                for r in csv.DictReader(f):
                    k = r['Kernel_Name']
                    if filt not in k:
                        continue
                    c = r['Counter_Name']
                    tab[k][(d, c)] += float(r['Counter_Value'])
                    disp[k][d].add(r['Dispatch_Id'])
    for k in sorted(tab):
        print(f'== {k[:140]}')
        for d in dirs:
            n = len(disp[k][d])
            if not n:
                continue
            grbm = tab[k].get((d, 'GRBM_GUI_ACTIVE'))
            cyc = grbm / n / 8 if grbm else None
            for (dd, c), v in sorted(tab[k].items()):
                if dd != d:
                    continue
                per = v / n
                extra = ''
                if cyc and c != 'GRBM_GUI_ACTIVE':
                    extra = f'   /kernel-cycle {per / cyc:10.3f}   /SIMD-cycle {per / cyc / 1024:8.4f}'
                print(f'  {c:32s} {per:16.4g}{extra}')
            if cyc:
                print(f'  {"kernel cycles (GRBM/8)":32s} {cyc:16.4g}')


if __name__ == '__main__':
    main()
