"""Per-launch comparison of two rocprofv3 kernel traces of the same program (tools/debug/trace_ab.sh): dispatches are
matched by order within (kernel name, grid), and the mean duration of each (name, grid, occurrence-class) is printed for
both traces.  usage: trace_cmp.py A/run_kernel_trace.csv B/run_kernel_trace.csv [name-substring]"""
import csv
import re
import sys
from collections import defaultdict


def load(p):
    rows = list(csv.DictReader(open(p)))
    out = defaultdict(list)
    for r in rows:
        name = re.sub(r'\(.*', '', r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', ''))[:60]
        key = (name, int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), int(r['Grid_Size_Z']))
        out[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
flt = sys.argv[3] if len(sys.argv) > 3 else ''
tot_a = tot_b = 0.0
for k in sorted(set(a) | set(b), key=lambda k: -sum(a.get(k, [0]))):
    if flt not in k[0]:
        continue
    da, db = a.get(k, []), b.get(k, [])
    # drop the first third (warm-up) when there are enough launches
    sa, sb = da[len(da) // 3:] or da, db[len(db) // 3:] or db
    ma = sum(sa) / max(len(sa), 1)
    mb = sum(sb) / max(len(sb), 1)
    tot_a += ma * len(sa)
    tot_b += mb * len(sb)
    print(f'{k[0]:60s} wg={k[1]:6d} z={k[2]:3d} n={len(sa):4d}  A {ma:8.1f}  B {mb:8.1f}  {100 * (mb / ma - 1) if ma else 0:+6.1f}%')
print(f'total (post-warm-up launches) A {tot_a / 1e3:.2f} ms  B {tot_b / 1e3:.2f} ms')
