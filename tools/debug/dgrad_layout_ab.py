"""A/B: the bench step's input-gradient GEMMs in the dgrad layout (B = W [N, K], row-contraction reads) against the
same products in the forward layout on a transposed weight copy (B = Wᵀ [K, N], K-contiguous): interleaved rounds in
one process, median µs per launch, and a bit-identity check of the two outputs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd')]
import torch  # noqa: E402
from cmhar import _lib as L  # noqa: E402
from cmhar import kernels as K  # noqa: E402

M = 32 * 1568
SHAPES = [('qkv', 2304, 768, False), ('out', 768, 768, False), ('fc1', 3072, 768, False), ('fc2', 768, 3072, True),
          ('kv_t0', 1536, 768, False)]


def main(rounds=7, reps=5):
    torch.manual_seed(0)
    res = {}
    for name, n, k, mulaux in SHAPES:
        dy = torch.randn(M, n, device='cuda').bfloat16()
        w = (torch.randn(n, k, device='cuda') * 0.03).bfloat16()
        wt = w.t().contiguous()
        aux = torch.randn(M, k, device='cuda').bfloat16() if mulaux else None
        o1 = torch.empty(M, k, dtype=torch.bfloat16, device='cuda')
        o0 = torch.empty_like(o1)
        kw = dict(act=L.ACT_MULAUX, aux_in=aux) if mulaux else {}
        fns = {'dgrad': lambda: K.gemm(1, dy, w, o1, **kw), 'fwd_wt': lambda: K.gemm(0, dy, wt, o0, **kw)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        same = torch.equal(o0, o1)
        times = {k_: [] for k_ in fns}
        for _ in range(rounds):
            for key, f in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    f()
                e1.record()
                e1.synchronize()
                times[key].append(1000 * e0.elapsed_time(e1) / reps)
        med = {key: sorted(v)[len(v) // 2] for key, v in times.items()}
        res[name] = med
        print(f'{name:6s} M={M} N={k} K={n}{" mulaux" if mulaux else ""}: dgrad {med["dgrad"]:.1f} us, '
              f'fwd(Wt) {med["fwd_wt"]:.1f} us, bit-identical {same}', flush=True)
        del dy, w, wt, aux, o0, o1
        torch.cuda.empty_cache()
    per_step = {key: sum(res[s][key] * (11 if s != 'kv_t0' else 1) for s in res) for key in ('dgrad', 'fwd_wt')}
    print('per step (11 layers + token-0 K|V):', {k_: round(v / 1000, 3) for k_, v in per_step.items()}, 'ms')


if __name__ == '__main__':
    main()
