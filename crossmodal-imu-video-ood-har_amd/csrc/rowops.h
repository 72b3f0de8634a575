// Row-level device routines shared by the stand-alone kernels and the fused IMU encoder kernel (imu_fused.hip), so
// that both compile the same arithmetic: the fused forward is bit-identical to the chain of separate launches.
// Every routine turns FP contraction off (CMHAR_NO_CONTRACT) and writes its fused multiply-adds as explicit fmaf:
// with contraction left to the backend, the same source inlined into two kernels was contracted differently (one
// o·α + p·v pair of the attention row became mul + add in the fused kernel, measured 1-ulp differences).  The
// explicit fmaf sites are exactly where the stand-alone kernels' previous build contracted (read off their ISA), so
// their numerics are unchanged — g1 / g4 / g6 pin them to the reference, and the IMU encoder's post-LN backward
// turns 1-ulp changes of its LayerNorm / attention arithmetic into ~1e-3 relative moves of some bias gradients.
#define CMHAR_NO_CONTRACT _Pragma("clang fp contract(off)")
#pragma once
#include "common.h"

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Attention-prob dropout (nn.MultiheadAttention semantics): keep (bh, q, k) iff hash >= p * 2^32, scale 1/(1-p).
__device__ __forceinline__ unsigned hash4(unsigned long long seed, unsigned a, unsigned b, unsigned c) {
  unsigned long long x = seed ^ (0x9E3779B97F4A7C15ull * (a + 1)) ^ (0xC2B2AE3D27D4EB4Full * (b + 1)) ^
                         (0x165667B19E3779F9ull * (c + 1));
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (unsigned)x;
}
__device__ __forceinline__ float drop_scale(unsigned long long seed, float p, unsigned bh, unsigned q, unsigned k) {
  if (p <= 0.f) return 1.f;
  const float u = (float)hash4(seed, bh, q, k) * 2.3283064365386963e-10f;
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

constexpr int LN_MAXPER = 16;   // LayerNorm columns per lane: N <= 1024

// One LayerNorm row by one wave (lane owns columns lane + 64i): y = LN(a + drop(b)) with gamma/beta, h_out
// (optional) = a + drop(b).  a, b, h_out, y point at the row; `row` is the global row index of the dropout hash.
template <typename T>
__device__ __forceinline__ void ln_row_fwd(int lane, long row, int N, const T* __restrict__ a, const T* __restrict__ b,
                                           float pdrop, unsigned long long seed, T* __restrict__ h_out,
                                           T* __restrict__ y, const float* __restrict__ gamma,
                                           const float* __restrict__ beta, float eps, float& mu_out, float& r_out) {
  CMHAR_NO_CONTRACT
  float v[LN_MAXPER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXPER; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < N) {
      float x = to_f<T>(a[c]);
      if (b) x = fmaf(to_f<T>(b[c]), drop_mask(seed, pdrop, row, c), x);
      v[i] = x;
      s += x;
    }
  }
  const float mu = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXPER; ++i) {
    const int c = lane + 64 * i;
    if (c < N) { const float d = v[i] - mu; q = fmaf(d, d, q); }
  }
  const float r = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXPER; ++i) {
    const int c = lane + 64 * i;
    if (c < N) {
      if (h_out) h_out[c] = from_f<T>(v[i]);
      y[c] = from_f<T>(fmaf((v[i] - mu) * r, gamma[c], beta[c]));
    }
  }
  mu_out = mu;
  r_out = r;
}

// Exact-fp32 attention of one query row over kn keys (online softmax in natural-log units, prob dropout): keys
// k0 .. k0+kn-1 at sK[kk*ldk + d], values at sV[kk*ldv + d]; qv carries the softmax scale.
template <int D>
__device__ __forceinline__ void attn_row_f32(const float (&qv)[D], float (&o)[D], float& m, float& l,
                                             const float* sK, int ldk, const float* sV, int ldv, int kn,
                                             unsigned long long seed, float pdrop, unsigned bh, int qq, int k0) {
  CMHAR_NO_CONTRACT
  for (int kk = 0; kk < kn; ++kk) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) s = fmaf(qv[d], sK[kk * ldk + d], s);
    const float mn = fmaxf(m, s);
    const float alpha = __expf(m - mn);
    const float p = __expf(s - mn);
    l = fmaf(l, alpha, p);
    const float pd = p * drop_scale(seed, pdrop, bh, qq, k0 + kk);
    // the stand-alone kernel's previous build fused all but the last two columns (d = D-2, D-1: separately rounded
    // o·α + p·v) — kept exactly, g1 pins this path to the reference
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float pv = pd * sV[kk * ldv + d];
      o[d] = d < D - 2 ? fmaf(o[d], alpha, pv) : o[d] * alpha + pv;
    }
    m = mn;
  }
}

// LayerNorm backward of one row by one wave: dy (pd) and the normalised input h (ph) per lane column (lane + 64i,
// zero past N), row mean / rstd → gx = rstd·(g − mean(g) − x̂·mean(g·x̂)) with g = dy·γ (before any residual add);
// ag / ab accumulate the row's dγ = dy·x̂ and dβ = dy terms.
template <int MP>
__device__ __forceinline__ void ln_row_bwd(int lane, int N, const float (&pd)[MP], const float (&ph)[MP], float mu,
                                           float r, const float* __restrict__ gamma, float (&ag)[MP], float (&ab)[MP],
                                           float (&gx)[MP]) {
  CMHAR_NO_CONTRACT
  float xh[MP], g[MP];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MP; ++i) {
    const int c = lane + 64 * i;
    xh[i] = 0.f;
    g[i] = 0.f;
    if (c < N) {
      const float d = pd[i];
      xh[i] = (ph[i] - mu) * r;
      g[i] = d * gamma[c];
      ag[i] = fmaf(d, xh[i], ag[i]);
      ab[i] += d;
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
  }
  s1 = wave_sum(s1) / N;
  s2 = wave_sum(s2) / N;
#pragma unroll
  for (int i = 0; i < MP; ++i) gx[i] = r * fmaf(-xh[i], s2, g[i] - s1);
}

// Exact-fp32 attention backward, dQ side: one query row (qv = q·scale, g = dO row, L = its natural-log LSE, delta =
// rowsum(dO∘O)) over kn keys at sK / sV; dq accumulates Σ ds·k (the caller applies the final ·scale).
template <int D>
__device__ __forceinline__ void attn_row_dq_f32(const float (&qv)[D], const float (&g)[D], float L, float delta,
                                                float (&dq)[D], const float* sK, int ldk, const float* sV, int ldv,
                                                int kn, unsigned long long seed, float pdrop, unsigned bh, int qq,
                                                int k0) {
  CMHAR_NO_CONTRACT
  for (int kk = 0; kk < kn; ++kk) {
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) { s = fmaf(qv[d], sK[kk * ldk + d], s); dp = fmaf(g[d], sV[kk * ldv + d], dp); }
    const float p = __expf(s - L);
    const float ds = p * fmaf(dp, drop_scale(seed, pdrop, bh, qq, k0 + kk), -delta);
#pragma unroll
    for (int d = 0; d < D; ++d) dq[d] = fmaf(ds, sK[kk * ldk + d], dq[d]);
  }
}

// dK / dV side: one key row (kv, vv) over qn query rows q0.. at sQ (times qs: the staged or on-the-fly softmax
// scale) and sG (dO), with their LSE Ls and delta Ds.
template <int D>
__device__ __forceinline__ void attn_row_dkdv_f32(const float (&kv)[D], const float (&vv)[D], float (&dk)[D],
                                                  float (&dv)[D], const float* sQ, int ldq, float qs, const float* sG,
                                                  int ldg, const float* Ls, const float* Ds, int qn,
                                                  unsigned long long seed, float pdrop, unsigned bh, int q0, int kk) {
  CMHAR_NO_CONTRACT
  for (int qi = 0; qi < qn; ++qi) {
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      s = fmaf(sQ[qi * ldq + d] * qs, kv[d], s);
      dp = fmaf(sG[qi * ldg + d], vv[d], dp);
    }
    const float p = __expf(s - Ls[qi]);
    const float ms = drop_scale(seed, pdrop, bh, q0 + qi, kk);
    const float ds = p * fmaf(dp, ms, -Ds[qi]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      dv[d] = fmaf(p * ms, sG[qi * ldg + d], dv[d]);
      dk[d] = fmaf(ds, sQ[qi * ldq + d] * qs, dk[d]);
    }
  }
}
