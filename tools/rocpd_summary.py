"""Summarise a rocprofv3 SQLite (.db) kernel trace: per-kernel calls, total / average duration, share."""
import sqlite3
import sys


def summary(path, top=30):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = 'kernel_name' if 'kernel_name' in cols else ('name' if 'name' in cols else None)
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start) from kernels "
                     f"group by {name_col} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = [f'{"kernel":100s} {"calls":>6s} {"total_ms":>10s} {"avg_us":>10s} {"pct":>6s}']
    for n, cnt, s, a in rows[:top]:
        out.append(f'{n[:100]:100s} {cnt:6d} {s / 1e6:10.3f} {a / 1e3:10.2f} {100 * s / tot:6.2f}')
    out.append(f'{"TOTAL":100s} {sum(r[1] for r in rows):6d} {tot / 1e6:10.3f}')
    # GPU busy time: union of all kernel intervals (streams overlap) vs the traced wall span
    iv = sorted(c.execute("select start, end from kernels").fetchall())
    busy, cur_s, cur_e = 0, None, None
    for a, b in iv:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        busy += cur_e - cur_s
        span = iv[-1][1] - iv[0][0]
        out.append(f'GPU busy (union of kernel intervals) {busy / 1e6:.3f} ms of {span / 1e6:.3f} ms span '
                   f'({100 * busy / span:.1f} %)')
    # steady-state steps: windows between consecutive optimizer launches (the last kernel of a training step)
    ends = [r[0] for r in c.execute(f"select end from kernels where {name_col} like '%mt_adamw%' order by end")]
    if len(ends) >= 3:
        lo, hi = ends[1], ends[-1]
        w = [(max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi]
        wb, ce, cs = 0, None, None
        for a, b in sorted(w):
            if ce is None or a > ce:
                if ce is not None:
                    wb += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        wb += ce - cs
        n = len(ends) - 2
        out.append(f'steady state: {n} steps, {(hi - lo) / 1e6 / n:.3f} ms/step wall, '
                   f'{wb / 1e6 / n:.3f} ms/step GPU busy ({100 * wb / (hi - lo):.1f} %)')
    return '\n'.join(out)


if __name__ == '__main__':
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30))
