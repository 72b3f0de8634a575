"""MFMA-pipe utilisation per kernel from one rocprofv3 PMC pass over a bench command:
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --kernel-trace --output-format csv \
        -d D -o run -- python bench.py ...
    python tools/pmc_mfma.py D OUT.json [COMMIT] [CMD]
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every SIMD (MI355X_MICROARCH.md: 32 x N for
v_mfma_f32_32x32x16_bf16); GRBM_GUI_ACTIVE is summed over the 8 XCDs, so GRBM/8 is the kernel's cycle count at the
clock it ran (the guide's DVFS note).  util = BUSY / (4 SIMDs x 256 CUs x GRBM/8).  With the kernel trace the
effective clock GRBM/8 / duration is reported too."""
import collections
import csv
import glob
import json
import sys


def main():
    busy = collections.defaultdict(float)
    grbm = collections.defaultdict(float)
    nmfma = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for fn in glob.glob(f'{sys.argv[1]}/**/*counter_collection.csv', recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                k, c, v = r['Kernel_Name'], r['Counter_Name'], float(r['Counter_Value'])
                disp[k].add(r['Dispatch_Id'])
                if c == 'SQ_VALU_MFMA_BUSY_CYCLES':
                    busy[k] += v
                elif c == 'GRBM_GUI_ACTIVE':
                    grbm[k] += v
                elif c == 'SQ_INSTS_MFMA':
                    nmfma[k] += v
    for fn in glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                dur[r['Kernel_Name']] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    out = {}
    for k in disp:
        n = len(disp[k])
        rec = {'dispatches': n, 'mfma_busy_cycles_per_launch': busy[k] / n, 'grbm_gui_active_per_launch': grbm[k] / n,
               'mfma_insts_per_launch': nmfma[k] / n,
               'mfma_util': busy[k] / (grbm[k] / 8 * 256 * 4) if grbm[k] else None}
        if dur.get(k):
            rec['effective_clock_ghz'] = round(grbm[k] / 8 / dur[k] / 1e9, 3)
        out[k] = rec
    with open(sys.argv[2], 'w') as f:
        json.dump({'note': 'mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (4 x 256 x GRBM_GUI_ACTIVE / 8) per dispatch '
                           '(one rocprofv3 --pmc pass of the same bench command)',
                   'commit': sys.argv[3] if len(sys.argv) > 3 else None,
                   'cmd': sys.argv[4] if len(sys.argv) > 4 else None, 'kernels': out}, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]['mfma_busy_cycles_per_launch'] * kv[1]['dispatches'])[:12]:
        u = v['mfma_util']
        print(f"util {u if u is None else round(u, 3)!s:>6}  clk {v.get('effective_clock_ghz')}  x{v['dispatches']:4d}  "
              f"{k[:100]}")


if __name__ == '__main__':
    main()
