"""Reference and error bound for the bf16 flash-attention kernels (csrc/attention.hip), shared by the kernel tests and
the production-shape test.

For the same operands it computes two things per output (O, dQ, dK, dV), chunked over clips so that the B·H·L² score
matrices of the production shape (B = 32, H = 12, L = 1568) never exist at once:
* the fp32 torch autograd reference: softmax(Q·Kᵀ·scale)·V and its gradients;
* the same algorithm with the kernel's bf16 roundings emulated (`oracle/cpu_model._FlashBF16`: P rounded before P·V
  and Pᵀ·dO, dS rounded before dS·K and dSᵀ·Q, δ from the bf16-stored O) and every output rounded to bf16 as the kernel
  stores it.
The bound a test applies: the kernel's error against the fp32 reference ≤ 3 × the emulation's error + 1e-3 (global
relative L2 norm per tensor, accumulated over the chunks).  A kernel error on top of bf16 rounding — a wrong tile, a
missed rescale, a tail row — shows as a multiple of the emulated error; summation order and exp2's last bit do not."""
import torch

from oracle.cpu_model import _FlashBF16

NAMES = ('o', 'dq', 'dk', 'dv')


def _heads(t, b, L, H, D):
    return t.float().reshape(b, L, H, D).transpose(1, 2).contiguous()


def _rows(t, b, L, H, D):
    return t.transpose(1, 2).reshape(b * L, H * D)


def flash_pair(q, k, v, do, *, b, H, Lq, Lk, D, scale):
    """fp32 reference and bf16-rounding emulation for b clips: dict name → (ref, emu), each [b·L, H·D] fp32.
    q, v, do: bf16 (or bf16-valued) [b·L, H·D]; k: the key the model means (for pre-scaled keys kp / c in fp32)."""
    qh, kh, vh = (_heads(t, b, Lx, H, D) for t, Lx in ((q, Lq), (k, Lk), (v, Lk)))
    doh = _heads(do, b, Lq, H, D)
    out = {}
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (qh, kh, vh))
    o = torch.softmax(qr @ kr.transpose(-1, -2) * scale, -1) @ vr
    g = torch.autograd.grad(o, (qr, kr, vr), doh)
    ref = (o.detach(),) + g
    qe, ke, ve = (t.clone().requires_grad_(True) for t in (qh, kh, vh))
    oe = _FlashBF16.apply(qe, ke, ve, scale)
    ge = torch.autograd.grad(oe, (qe, ke, ve), doh)
    emu = tuple(t.detach().bfloat16().float() for t in (oe,) + ge)
    for n, r, e in zip(NAMES, ref, emu):
        L_ = Lq if n in ('o', 'dq') else Lk
        out[n] = (_rows(r, b, L_, H, D), _rows(e, b, L_, H, D))
    return out


class FlashErrors:
    """Accumulates ‖got − ref‖², ‖emu − ref‖², ‖ref‖² per output (optionally on a row sub-range per clip)."""

    def __init__(self):
        self.s = {n: [0.0, 0.0, 0.0] for n in NAMES}

    def add(self, name, got, ref, emu):
        got, ref, emu = got.double(), ref.double(), emu.double()
        a = self.s[name]
        a[0] += (got - ref).pow(2).sum().item()
        a[1] += (emu - ref).pow(2).sum().item()
        a[2] += ref.pow(2).sum().item()

    def errors(self, name):
        g, e, r = self.s[name]
        r = max(r, 1e-300)
        return (g / r) ** 0.5, (e / r) ** 0.5

    def check(self, mult=3.0, floor=1e-3):
        msgs = []
        for n in NAMES:
            if self.s[n][2] == 0.0:
                continue
            g, e = self.errors(n)
            if not g <= mult * e + floor:
                msgs.append(f'{n}: kernel {g:.3e} > {mult} x emulated {e:.3e} + {floor}')
        assert not msgs, '; '.join(msgs)
        return {n: self.errors(n) for n in NAMES if self.s[n][2] > 0.0}


def check_flash(got, q, k, v, do, *, B, H, Lq, Lk, D, scale, chunk=None, row_ranges=None):
    """got: dict name → kernel output [B·L, H·D] (bf16).  Chunks of `chunk` clips (default: all at once).
    row_ranges: optional dict 'q' / 'k' → first row (per clip) of a sub-region checked on its own as well (the ragged
    tails).  Returns the per-output (kernel, emulated) errors of the whole tensors."""
    chunk = chunk or B
    whole, parts = FlashErrors(), FlashErrors()
    for b0 in range(0, B, chunk):
        b = min(chunk, B - b0)
        sl = lambda t, L_: t[b0 * L_:(b0 + b) * L_]      # noqa: E731
        pair = flash_pair(sl(q, Lq), sl(k, Lk), sl(v, Lk), sl(do, Lq), b=b, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
        for n, (ref, emu) in pair.items():
            L_ = Lq if n in ('o', 'dq') else Lk
            g = sl(got[n], L_).float()
            whole.add(n, g, ref, emu)
            if row_ranges is not None:
                r0 = row_ranges['q' if n in ('o', 'dq') else 'k']
                cut = lambda t: t.view(b, L_, -1)[:, r0:]      # noqa: E731
                parts.add(n, cut(g), cut(ref), cut(emu))
        del pair
    res = whole.check()
    if row_ranges is not None:
        parts.check()
    return res
