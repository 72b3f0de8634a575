"""R3D-18 bf16 path vs the fp32 oracle and its bf16-storage emulation, layer by layer.

For every conv unit (stem, conv1, downsample, conv2 of each block): rel error of the GPU's stored conv output z and
unit output y against the fp32 oracle, and the emulation's error against the same; then per-parameter gradient
errors (GPU vs fp32, emulation vs fp32) sorted by their ratio, and the CrossModal loss at the DP worker's geometry.
Prints one table; a unit whose GPU error exceeds 3x the emulation's is where a kernel adds error."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'), os.path.join(REPO, 'tests')]
import torch  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def cl(t):      # NCDHW → [rows, C] (the HIP path's NDHWC rows)
    return t.permute(0, 2, 3, 4, 1).reshape(-1, t.shape[1])


def main(B=4, T=4, S=48):
    from cmhar.r3d import R3D18, _forward_impl, run_r3d
    from oracle.r3d_cpu import BF16, r3d18_features
    torch.manual_seed(2)
    m = R3D18(None, compute_dtype='bf16')
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm3d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    video = torch.randn(B, T, 3, S, S)
    R = torch.randn(B, 512)

    def oracle(hooks):
        sd_p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and 'running' not in k else v.clone())
                for k, v in sd.items()}
        trace = []
        ref = r3d18_features(sd_p, video.transpose(1, 2), training=True, trace=trace, **hooks)
        (ref * R).sum().backward()
        return sd_p, trace, ref

    sd32, tr32, ref32 = oracle({})
    sdq, trq, refq = oracle(BF16)
    m = m.cuda().train()
    with torch.no_grad():
        m2 = R3D18(None, compute_dtype='bf16')
        m2.load_state_dict(sd)
        m2 = m2.cuda().train()
        _, st = _forward_impl(m2, video.cuda(), True, save=True)
    units = st[0]
    print(f'{"unit":>4} {"rows":>7} {"C":>4} | z: gpu/fp32  emul/fp32 | y: gpu/fp32  emul/fp32')
    for i, (u, (z32, y32), (zq, yq)) in enumerate(zip(units, tr32, trq)):
        M = u.z.shape[0]
        zg, yg = u.z[:M].float(), u.y[:M].float()
        print(f'{i:4d} {M:7d} {zg.shape[1]:4d} | {rel(zg, cl(z32)):.2e}  {rel(cl(zq), cl(z32)):.2e} | '
              f'{rel(yg, cl(y32)):.2e}  {rel(cl(yq), cl(y32)):.2e}')
    feat = run_r3d(m, video.cuda(), True)
    (feat * R.cuda()).sum().backward()
    print(f'features: gpu {rel(feat, ref32):.2e} emul {rel(refq, ref32):.2e}')
    rows = []
    for k, p in m.named_parameters():
        eg, ep = rel(p.grad, sd32[k].grad), rel(sdq[k].grad, sd32[k].grad)
        rows.append((eg / max(ep, 1e-12), eg, ep, k))
    rows.sort(reverse=True)
    print('grads: ratio gpu/emul, gpu err, emul err, param (worst 12)')
    for r in rows[:12]:
        print(f'  {r[0]:6.2f} {r[1]:.2e} {r[2]:.2e} {r[3]}')
    print('max gpu err', max(r[1] for r in rows), 'max emul', max(r[2] for r in rows))


if __name__ == '__main__':
    main()
