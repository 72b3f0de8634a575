"""Per-kernel summary of a rocprofv3 --kernel-trace CSV run: calls, total / average duration, share, plus the GPU-busy
union and the per-step wall time of the last N steps (steps delimited by the AdamW kernel).
python tools/kstats.py DIR [steps_in_run]
With CMHAR_KSTATS_CONTEXT=pattern[,pattern...]: per steady-state step, which kernels launch right before / after the
kernels whose names contain a pattern (small torch kernels: who issues them)."""
import os
import collections
import csv
import glob
import sys


def main():
    path = sys.argv[1]
    rows = []
    for fn in glob.glob(f'{path}/**/*kernel_trace.csv', recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    agg = collections.defaultdict(lambda: [0, 0])
    for a, b, n in rows:
        agg[n][0] += 1
        agg[n][1] += b - a
    tot = sum(v[1] for v in agg.values())
    print(f'{"kernel":100s} {"calls":>6s} {"total_ms":>10s} {"avg_us":>10s} {"pct":>6s}')
    for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f'{n[:100]:100s} {c:6d} {s / 1e6:10.3f} {s / c / 1e3:10.2f} {100 * s / tot:6.2f}')
    print(f'{"TOTAL":100s} {len(rows):6d} {tot / 1e6:10.3f}')
    # steady state: AdamW kernel ends delimit steps
    ends = [b for a, b, n in rows if 'mt_adamw_kernel' in n]
    if len(ends) >= 3:
        k = len(ends) - 1
        span = ends[-1] - ends[1]
        iv = [(a, b) for a, b, n in rows if ends[1] <= a < ends[-1]]
        busy, cs, ce = 0, None, None
        for a, b in sorted(iv):
            if ce is None or a > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        if ce is not None:
            busy += ce - cs
        n = k - 1
        print(f'steady state: {n} steps, {span / n / 1e6:.3f} ms/step wall, {busy / n / 1e6:.3f} ms/step GPU busy '
              f'({100 * busy / span:.1f} %)')
        gaps = [iv_b[0] - iv_a[1] for iv_a, iv_b in zip(sorted(iv), sorted(iv)[1:]) if iv_b[0] > iv_a[1]]
        print(f'inter-kernel gaps: {len(gaps) / n:.0f} per step, {sum(gaps) / n / 1e6:.3f} ms/step')
        # where the idle time sits: gaps of the steady-state steps by (previous kernel -> next kernel), summed
        st = sorted((a, b, nm) for a, b, nm in rows if ends[1] <= a < ends[-1])
        by = collections.defaultdict(lambda: [0, 0])
        ce, cn = None, None
        for a, b, nm in st:
            if ce is not None and a > ce:
                key = (cn[:60], nm[:60])
                by[key][0] += 1
                by[key][1] += a - ce
            if ce is None or b > ce:
                ce, cn = b, nm
        print('largest idle intervals by (kernel before -> kernel after), per step:')
        for (x, y), (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1])[:15]:
            print(f'  {t / n / 1e3:8.1f} us  x{c / n:5.1f}  {x}  ->  {y}')
        for pat in filter(None, os.environ.get('CMHAR_KSTATS_CONTEXT', '').split(',')):
            ctx = collections.Counter()
            for i, (a, b, nm) in enumerate(st):
                if pat in nm:
                    prev = st[i - 1][2][:70] if i else '-'
                    nxt = st[i + 1][2][:70] if i + 1 < len(st) else '-'
                    ctx[(prev, nxt)] += 1
            print(f'context of "{pat}" per step ({sum(ctx.values()) / n:.1f} launches):')
            for (x, y), c in ctx.most_common(25):
                print(f'  x{c / n:5.1f}  {x}  ->  *  ->  {y}')


if __name__ == '__main__':
    main()
