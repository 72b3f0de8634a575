"""Per-launch HBM traffic of the step's weight-gradient GEMMs (dW = dYᵀX over M = 50176 tokens), one shape at a time:
    run      python tools/debug/pmc_wgrad.py run            (under rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE)
    report   python tools/debug/pmc_wgrad.py report FETCH_DIR WRITE_DIR
Each shape is launched twice; the report lists every GEMM / reduce dispatch in order with its bytes against the
algorithmic dY + X reads + fp32 dW write (the split-K partial slabs are the difference's known part)."""
import csv
import glob
import os
import sys

SHAPES = [('qkv', 2304, 768), ('out', 768, 768), ('fc1', 3072, 768), ('fc2', 768, 3072), ('embed', 768, 1536)]
T = 50176


def run():
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                    'crossmodal-imu-video-ood-har_amd'))
    from cmhar import kernels as K
    for name, n_out, n_in in SHAPES:
        x = torch.randn(T, n_in, device='cuda').bfloat16()
        dy = torch.randn(T, n_out, device='cuda').bfloat16()
        dw = torch.empty(n_out, n_in, device='cuda')
        for _ in range(2):
            K.gemm(2, dy, x, dw)
        torch.cuda.synchronize()
    print('done')


def report(fd, wd):
    def rows(d, cname):
        out = {}
        for fn in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
            for r in csv.DictReader(open(fn)):
                if r['Counter_Name'] == cname:
                    k = int(r['Dispatch_Id'])
                    nm, v = out.get(k, (r['Kernel_Name'], 0.0))
                    out[k] = (nm, v + float(r['Counter_Value']) * 1024)
        return out
    f, w = rows(fd, 'FETCH_SIZE'), rows(wd, 'WRITE_SIZE')
    fl = [v for k, v in sorted(f.items()) if 'gemm' in v[0] or 'reduce' in v[0]]
    wl = [v for k, v in sorted(w.items()) if 'gemm' in v[0] or 'reduce' in v[0]]
    i = 0
    for name, n_out, n_in in SHAPES:
        alg = T * (n_out + n_in) * 2 + n_out * n_in * 4
        for rep in range(2):
            while i < len(fl) and 'gemm' not in fl[i][0]:
                i += 1
            if i >= len(fl):
                return
            g = (2 * fl[i][1], wl[i][1])
            red = (2 * fl[i + 1][1], wl[i + 1][1]) if i + 1 < len(fl) and 'reduce' in fl[i + 1][0] else (0.0, 0.0)
            print(f'{name:6s} gemm fetch {g[0] / 1e6:7.1f} MB write {g[1] / 1e6:6.1f} MB | reduce fetch {red[0] / 1e6:6.1f} '
                  f'write {red[1] / 1e6:5.1f} | algorithmic {alg / 1e6:6.1f} MB | gemm/alg {(g[0] + g[1]) / alg:4.2f}')
            i += 2 if red[0] else 1


if __name__ == '__main__':
    run() if sys.argv[1] == 'run' else report(sys.argv[2], sys.argv[3])
