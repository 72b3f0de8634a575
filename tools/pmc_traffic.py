"""HBM traffic per kernel launch from two rocprofv3 PMC passes over the same bench command:
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d D1 -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d D2 -o run -- python bench.py ...
    python tools/pmc_traffic.py D1 D2 OUT.json [COMMIT] [CMD]
FETCH_SIZE and WRITE_SIZE are in KB (1024 B).  gfx950 correction (MI355X_MICROARCH.md § HBM): FETCH_SIZE reports
exactly half of the bytes of wide coalesced reads (128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Infinity-Cache hits are counted by these memory-side counters."""
import collections
import csv
import glob
import json
import sys


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for fn in glob.glob(f'{path}/**/*counter_collection.csv', recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r['Counter_Name'] != counter:
                    continue
                tot[r['Kernel_Name']] += float(r['Counter_Value'])
                disp[r['Kernel_Name']].add(r['Dispatch_Id'])
    return {k: (tot[k], len(disp[k])) for k in tot}


def main():
    fetch = per_kernel(sys.argv[1], 'FETCH_SIZE')
    write = per_kernel(sys.argv[2], 'WRITE_SIZE')
    out = {}
    for k in set(fetch) | set(write):
        fk, fn = fetch.get(k, (0.0, 0))
        wk, wn = write.get(k, (0.0, 0))
        n = max(fn, wn, 1)
        out[k] = {'dispatches': n, 'fetch_bytes_per_launch': 2 * 1024 * fk / max(fn, 1),
                  'write_bytes_per_launch': 1024 * wk / max(wn, 1)}
        out[k]['hbm_bytes_per_launch'] = out[k]['fetch_bytes_per_launch'] + out[k]['write_bytes_per_launch']
    with open(sys.argv[3], 'w') as f:
        json.dump({'note': 'FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB=1024 B, per dispatch; '
                           'source: two rocprofv3 --pmc passes of the same bench command',
                   'commit': sys.argv[4] if len(sys.argv) > 4 else None,
                   'cmd': sys.argv[5] if len(sys.argv) > 5 else None, 'kernels': out}, f,
                  indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'] * kv[1]['dispatches'])[:12]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch (fetch {v['fetch_bytes_per_launch'] / 1e6:8.1f}, "
              f"write {v['write_bytes_per_launch'] / 1e6:8.1f})  x{v['dispatches']:4d}  {k[:100]}")


if __name__ == '__main__':
    main()
