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
    return '\n'.join(out)


if __name__ == '__main__':
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30))
