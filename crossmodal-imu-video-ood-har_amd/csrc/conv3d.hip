// R3D-18 video backbone support (north_star extension "VideoEncoder 3D-conv/R3D"; SURVEY §8 a11 — the reference has no
// 3-D CNN, its CNN options are per-frame 2-D torchvision models, models.py:160-216).
//
// Activations live channels-last (NDHWC: [clips, T, H, W, C]) so that one output position's receptive field is
// kt·kh·kw contiguous C-vectors and a convolution is a GEMM over rows = output positions:
//   col[m, k] (k = ((it·kh + ih)·kw + iw)·C + c, zero-padded to Kp)  →  y[m, co] = col[m, :] · Wp[co, :]ᵀ
// on the bf16 MFMA GEMM (gemm_bf16.hip, layout 0); dgrad = dy·Wp (layout 1) gathered back by col2im; wgrad =
// dyᵀ·col (layout 2).  BatchNorm3d (training batch statistics, eps/momentum as nn.BatchNorm3d) is a two-level
// deterministic column reduction over the [M, C] view plus an apply pass that fuses the residual add and ReLU of
// torchvision's BasicBlock; its backward fuses the ReLU mask and emits the residual-branch gradient.
#include "common.h"

namespace {

// Register-prefetched operand loads of padding / out-of-range slots read a valid address and are zeroed when they
// are written to LDS, not when they are loaded: a select on a prefetched load's result right after the load makes
// the compiler wait for that load there (s_waitcnt vmcnt(0) in the load phase, before the compute it was meant to
// overlap).  CMHAR_LATE_ZERO=0 (build flag): the select at the load (A/B builds).
// s_setprio(1) over a conv kernel's MFMA phase, so a CU's co-resident workgroup in its LDS-store phase does not
// take issue slots from it (nine-tap forward: R3D-18 layer 2 203.0 -> 196.9 us, layer 3 95.8 -> 92.2, A/B builds)
#ifndef CMHAR_ROWS3_PRIO
#define CMHAR_ROWS3_PRIO 1   // conv3d_fwd_rows3
#endif
#ifndef CMHAR_ROWS_PRIO
#define CMHAR_ROWS_PRIO 0    // conv3d_fwd_rows
#endif
#ifndef CMHAR_IGEMM_PRIO
#define CMHAR_IGEMM_PRIO 0   // conv3d_fwd_igemm
#endif
#ifndef CMHAR_LATE_ZERO
#define CMHAR_LATE_ZERO 1
#endif
constexpr bool kLateZero = CMHAR_LATE_ZERO != 0;
__device__ __forceinline__ uint4_t zero_unless(bool ok, uint4_t v) { return ok ? v : uint4_t{0u, 0u, 0u, 0u}; }

template <typename T, int V> __device__ __forceinline__ void vload(const T* p, float* v) {
  if constexpr (V == 8) Vec8<T>::load(p, v);
  else for (int j = 0; j < V; ++j) v[j] = to_f<T>(p[j]);
}
template <typename T, int V> __device__ __forceinline__ void vstore(T* p, const float* v) {
  if constexpr (V == 8) Vec8<T>::store(p, v);
  else for (int j = 0; j < V; ++j) p[j] = from_f<T>(v[j]);
}
// conv epilogue output (8 bf16), non-temporal as the GEMM epilogues (R3D-18 step 1659 / 1662 -> 1672 / 1671 clips/s,
// tools/debug/lib_workload_ab.sh); CMHAR_CONV_NT=0: plain stores
#ifndef CMHAR_CONV_NT
#define CMHAR_CONV_NT 1
#endif
__device__ __forceinline__ void zstore8(bf16* p, const float* v) {
  if (CMHAR_CONV_NT) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j];
    typedef int __attribute__((ext_vector_type(4))) i4;
    __builtin_nontemporal_store(__builtin_bit_cast(i4, r), (i4*)p);
  } else {
    Vec8<bf16>::store(p, v);
  }
}

struct Geom {
  int N, T, H, W, C;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int To, Ho, Wo, K, Kp;
};

// Rows are handled by groups of TPR threads (TPR = the power of two ≥ Kp/V, at most 256), so a row's output
// position is decomposed once per thread in 32-bit arithmetic and each thread writes V consecutive k of one tap
// (V = 8 when C % 8 == 0: a 16-B bf16 vector).
template <typename TI, typename TO, int V>
__global__ __launch_bounds__(256) void im2col3d_kernel(Geom g, int M, int tpr, const TI* __restrict__ x,
                                                       TO* __restrict__ col) {
  const int kv = g.Kp / V, rpb = 256 / tpr;
  const int sub = threadIdx.x / tpr, lane = threadIdx.x % tpr;
  for (int rb = blockIdx.x * rpb; rb < M; rb += gridDim.x * rpb) {
    const int row = rb + sub;
    if (row >= M) continue;
    int r = row;
    const int wo = r % g.Wo; r /= g.Wo;
    const int ho = r % g.Ho; r /= g.Ho;
    const int to = r % g.To;
    const int n = r / g.To;
    const int t0 = to * g.st - g.pt, h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
    TO* dst_row = col + (long)row * g.Kp;
    for (int j = lane; j < kv; j += tpr) {
      const int k = j * V;
      float v[V];
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = 0.f;
      if (k < g.K) {
        const int tap = k / g.C, c = k - tap * g.C;
        const int iw = tap % g.kw, ih = (tap / g.kw) % g.kh, it = tap / (g.kw * g.kh);
        const int ti = t0 + it, hi = h0 + ih, wi = w0 + iw;
        if (ti >= 0 && ti < g.T && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
          vload<TI, V>(x + ((((long)n * g.T + ti) * g.H + hi) * g.W + wi) * g.C + c, v);
        }
      }
      vstore<TO, V>(dst_row + k, v);
    }
  }
}

// Few input channels (the stem: C = 3, K = 441): each thread gathers 8 consecutive k of one row element by element
// (tap / channel advanced incrementally) and writes them as one 16-B vector — the column matrix is the traffic here.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col3d_vec_store_kernel(Geom g, int M, const TI* __restrict__ x,
                                                                 TO* __restrict__ col) {
  const int kv = g.Kp / 8;
  const long total = (long)M * kv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / kv), k0 = (int)(i - (long)row * kv) * 8;
    int r = row;
    const int wo = r % g.Wo; r /= g.Wo;
    const int ho = r % g.Ho; r /= g.Ho;
    const int to = r % g.To;
    const int n = r / g.To;
    const int t0 = to * g.st - g.pt, h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
    int tap = k0 / g.C, c = k0 - tap * g.C;
    int iw = tap % g.kw, ih = (tap / g.kw) % g.kh, it = tap / (g.kw * g.kh);
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float e = 0.f;
      if (k0 + q < g.K) {
        const int ti = t0 + it, hi = h0 + ih, wi = w0 + iw;
        if (ti >= 0 && ti < g.T && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
          e = to_f<TI>(x[((((long)n * g.T + ti) * g.H + hi) * g.W + wi) * g.C + c]);
      }
      v[q] = e;
      if (++c == g.C) {                       // next tap: (it, ih, iw) advance like an odometer
        c = 0;
        if (++iw == g.kw) { iw = 0; if (++ih == g.kh) { ih = 0; ++it; } }
      }
    }
    vstore<TO, 8>(col + (long)row * g.Kp + k0, v);
  }
}

// Gather form of col2im: every input element sums the (at most kt·kh·kw) column entries it fed, in tap order —
// deterministic, no atomics.  dx = Σ (+ dx_old when accumulate).  32-bit position arithmetic (host-checked).
template <typename T, int V>
__global__ __launch_bounds__(256) void col2im3d_kernel(Geom g, const T* __restrict__ dcol, T* __restrict__ dx,
                                                       int accumulate) {
  const int cv = g.C / V;
  const unsigned total = (unsigned)g.N * g.T * g.H * g.W * cv;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned pos = i / cv;
    const int c = (int)(i - pos * cv) * V;
    unsigned r = pos;
    const int w = r % g.W; r /= g.W;
    const int h = r % g.H; r /= g.H;
    const int t = r % g.T;
    const int n = r / g.T;
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int it = 0; it < g.kt; ++it) {
      const int tt = t + g.pt - it;
      if (tt < 0 || tt % g.st) continue;
      const int to = tt / g.st;
      if (to >= g.To) continue;
      for (int ih = 0; ih < g.kh; ++ih) {
        const int hh = h + g.ph - ih;
        if (hh < 0 || hh % g.sh) continue;
        const int ho = hh / g.sh;
        if (ho >= g.Ho) continue;
        for (int iw = 0; iw < g.kw; ++iw) {
          const int ww = w + g.pw - iw;
          if (ww < 0 || ww % g.sw) continue;
          const int wo = ww / g.sw;
          if (wo >= g.Wo) continue;
          const int row = ((n * g.To + to) * g.Ho + ho) * g.Wo + wo;
          float v[V];
          vload<T, V>(dcol + (long)row * g.Kp + ((it * g.kh + ih) * g.kw + iw) * g.C + c, v);
#pragma unroll
          for (int j = 0; j < V; ++j) acc[j] += v[j];
        }
      }
    }
    T* dst = dx + (long)pos * g.C + c;
    if (accumulate) {
      float o[V];
      vload<T, V>(dst, o);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += o[j];
    }
    vstore<T, V>(dst, acc);
  }
}

// The same gather for bf16 with 8 channels per thread, its loads issued together: per dimension the taps that can
// reach an input position are i0, i0 + s, … (i0 = (x + p) mod s, at most MT = ⌈k / s⌉ of them), so a fixed MT³
// nest enumerates the candidates in the tap order of col2im3d_kernel; each candidate's load goes through a buffer
// resource, an invalid one at an offset past the range (bit 31) that reads zero (+0 leaves the sum's bits unchanged),
// and all MT³ loads are in flight before the first add — the branches of col2im3d_kernel made each wait for the one
// before.  dcol stays within 2^31 bytes (host-checked).
template <int MT>
__global__ __launch_bounds__(256) void col2im3d_gather(Geom g, const bf16* __restrict__ dcol, bf16* __restrict__ dx,
                                                       int accumulate) {
  const int cv = g.C / 8;
  const unsigned total = (unsigned)g.N * g.T * g.H * g.W * cv;
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dcol, (short)0, (int)min((long)g.N * g.To * g.Ho * g.Wo * g.Kp * 2, 0x7fffffffL), 0x00020000);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned pos = i / cv;
    const int c = (int)(i - pos * cv) * 8;
    unsigned r = pos;
    const int w = r % g.W; r /= g.W;
    const int h = r % g.H; r /= g.H;
    const int t = r % g.T;
    const int n = r / g.T;
    const int it0 = (t + g.pt) % g.st, ih0 = (h + g.ph) % g.sh, iw0 = (w + g.pw) % g.sw;
    uint4_t v[MT * MT * MT];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b)
#pragma unroll
        for (int d = 0; d < MT; ++d) {
          const int it = it0 + a * g.st, ih = ih0 + b * g.sh, iw = iw0 + d * g.sw;
          const int to = (t + g.pt - it) / g.st, ho = (h + g.ph - ih) / g.sh, wo = (w + g.pw - iw) / g.sw;
          const bool ok = it < g.kt && ih < g.kh && iw < g.kw && t + g.pt - it >= 0 && h + g.ph - ih >= 0 &&
                          w + g.pw - iw >= 0 && to < g.To && ho < g.Ho && wo < g.Wo;
          const int e = (((n * g.To + to) * g.Ho + ho) * g.Wo + wo) * g.Kp + ((it * g.kh + ih) * g.kw + iw) * g.C + c;
          v[(a * MT + b) * MT + d] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(
              dr, (unsigned)(e * 2) | ((unsigned)!ok << 31), 0, 0));
        }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int q = 0; q < MT * MT * MT; ++q) {
      const bf16x8 b8 = __builtin_bit_cast(bf16x8, v[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)b8[j];
    }
    bf16* dst = dx + (long)pos * g.C + c;
    if (accumulate) {
      float o[8];
      Vec8<bf16>::load(dst, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    Vec8<bf16>::store(dst, acc);
  }
}

// ---- BatchNorm over the [M, C] channels-last view ----------------------------------------------------------------
// Column partial sums over a chunk of rows: each thread reads 8 consecutive channels of a row (one 16-B bf16
// vector), TPR = C/8 threads cover a row and the block's RPI = 256/TPR row slots are combined in a fixed order.
// mode 0: Σx; mode 1: Σ(x−mean)²; mode 2: Σg, Σg·x̂ with g = dy·act'(y) (relu 1: [y > 0]; relu 2 = ReLU6:
// [0 < y < 6]).  part: [2][nchunk][C].  C/8 need not divide 256: the 256 % TPR spare threads only add zeros.
// relu | BN_ZMASK: the unit had no residual input, so y = act(x̂·w + b) is recomputed from x in bn_cl_apply's exact
// arithmetic and rounding (bit-identical mask) instead of read: one M×C tensor less per pass.
constexpr int BN_ZMASK = 4;
// act'(y) ≠ 0 from the stored y: ReLU [y > 0] (+inf included, as torch's threshold_backward on the result), ReLU6
// [0 < y < 6]; NaN → 0.
__device__ __forceinline__ bool bn_y_on(float y, int relu) { return y > 0.f && ((relu & 3) != 2 || y < 6.f); }
// The same mask from the pre-activation v = fmaf((x − mean)·rstd, w, b) (bn_cl_apply's arithmetic), without the
// round trip y = T(clamp(v)): for bf16 storage T(v) of 0 < v ≤ 2^-134 is +0 (round to nearest even: 2^-134 is the
// tie between +0 and the smallest denormal 2^-133) and ReLU6's T(v) reaches 6 from v = 6 − 2^-6 on (the tie rounds
// to the even 6.0); fp32 storage keeps v.  NaN: the forward's clamp gives 0 → off, as here.
template <typename T>
__device__ __forceinline__ bool bn_act_on(float v, int relu) {
  constexpr bool B16 = sizeof(T) == 2;
  return v > (B16 ? 0x1p-134f : 0.f) && ((relu & 3) != 2 || v < (B16 ? 5.984375f : 6.f));
}
template <typename T, int MODE, bool ZM = false>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? 4 : 3) void bn_cl_partial(int M, int C, int rows_per_chunk, const T* __restrict__ x,
                                                     const T* __restrict__ y, const T* __restrict__ dy,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     int relu, float* __restrict__ part) {
  static_assert(MODE >= 0 && MODE <= 2 && (!ZM || MODE == 2), "modes 0 / 1 / 2; the z-mask in mode 2 only");
  __shared__ float s0[256][9], s1[256][9];
  const int tid = threadIdx.x;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int slot = tid / TPR, c0 = (tid % TPR) * 8;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(r0 + rows_per_chunk, M);
  const int rs0 = slot < RPI ? r0 + slot : r1;
  // ZM: a separate instantiation (the mask's w / b and the y loads never share registers); bf16: ≤ 128 VGPRs (launch
  // bounds), 4 waves per SIMD, the 1024 chunks of bn_chunks in one round; MODE compile-time: one loop body
  const bool ry = !ZM && MODE == 2 && relu;
  float mu[8], rs[8], a0[8], a1[8], ww[8], bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = MODE ? mean[c0 + j] : 0.f;
    rs[j] = MODE == 2 ? rstd[c0 + j] : 0.f;
    ww[j] = ZM ? w[c0 + j] : 0.f;
    bb[j] = ZM ? b[c0 + j] : 0.f;
    a0[j] = a1[j] = 0.f;
  }
  auto accum = [&](const float* v, const float* gv, const float* yv) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE == 0) {
        a0[j] += v[j];
      } else if (MODE == 1) {
        const float d = v[j] - mu[j];
        a0[j] = fmaf(d, d, a0[j]);
      } else {
        const float xh = (v[j] - mu[j]) * rs[j];
        const bool off = ZM ? !bn_act_on<T>(fmaf(xh, ww[j], bb[j]), relu) : relu && !bn_y_on(yv[j], relu);
        const float gj = off ? 0.f : gv[j];
        a0[j] += gj;
        a1[j] = fmaf(gj, xh, a1[j]);
      }
    }
  };
  // four row slots' loads in flight per thread (with 2–3 waves per SIMD one 16-B load per tensor left the kernel at
  // ~1.5 TB/s), accumulated in the same sequential row order as the one-row tail loop
  constexpr int UR = 4;
  int r = rs0;
  for (; r + (UR - 1) * RPI < r1; r += UR * RPI) {
    float v[UR][8], gv[UR][8], yv[UR][8];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long off = (long)(r + u * RPI) * C + c0;
      Vec8<T>::load(x + off, v[u]);
      if (MODE == 2) {
        Vec8<T>::load(dy + off, gv[u]);
        if (ry) Vec8<T>::load(y + off, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) accum(v[u], gv[u], yv[u]);
  }
  for (; r < r1; r += RPI) {
    const long off = (long)r * C + c0;
    float v[8], gv[8], yv[8];
    Vec8<T>::load(x + off, v);
    if (MODE == 2) {
      Vec8<T>::load(dy + off, gv);
      if (ry) Vec8<T>::load(y + off, yv);
    }
    accum(v, gv, yv);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { s0[tid][j] = a0[j]; s1[tid][j] = a1[j]; }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float b0 = 0.f, b1 = 0.f;
    for (int sl = 0; sl < RPI; ++sl) { b0 += s0[sl * TPR + c / 8][c % 8]; b1 += s1[sl * TPR + c / 8][c % 8]; }
    part[(long)blockIdx.x * C + c] = b0;
    if (MODE == 2) part[((long)gridDim.x + blockIdx.x) * C + c] = b1;
  }
}

// Combine the chunk partials (BN_FC columns per block, 256 / BN_FC chunk slots, fixed order) and finish the statistic.
// mode 0: mean;  mode 1: rstd (+ running stats, num_batches_tracked);  mode 2: db = Σg, dw = Σg·x̂.
// Each slot keeps BN_FU independent partial sums (BN_FU chunk loads in flight instead of one dependent chain; the
// kernel is load-latency bound: ≤ 512 KiB of partials), combined in a fixed order.
constexpr int BN_FC = 4, BN_FS = 256 / BN_FC, BN_FU = 4;
static_assert(BN_FU == 4, "the fixed-order combine below adds four partial sums");
__global__ __launch_bounds__(256) void bn_cl_final(int mode, long M, int C, int nchunk, const float* __restrict__ part,
                                                   float* __restrict__ mean, float* __restrict__ rstd,
                                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                                   long long* __restrict__ nbt, float momentum, float eps,
                                                   float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float s0[256], s1[256];
  const int tid = threadIdx.x, cl = tid % BN_FC, slot = tid / BN_FC;
  const int c = blockIdx.x * BN_FC + cl;
  float a0[BN_FU] = {}, a1[BN_FU] = {};
  if (c < C) {
    int k = slot;
    for (; k + (BN_FU - 1) * BN_FS < nchunk; k += BN_FU * BN_FS) {
#pragma unroll
      for (int u = 0; u < BN_FU; ++u) {
        a0[u] += part[(long)(k + u * BN_FS) * C + c];
        if (mode == 2) a1[u] += part[((long)nchunk + k + u * BN_FS) * C + c];
      }
    }
    for (; k < nchunk; k += BN_FS) {
      a0[0] += part[(long)k * C + c];
      if (mode == 2) a1[0] += part[((long)nchunk + k) * C + c];
    }
  }
  s0[tid] = (a0[0] + a0[1]) + (a0[2] + a0[3]);
  s1[tid] = (a1[0] + a1[1]) + (a1[2] + a1[3]);
  __syncthreads();
  if (slot || c >= C) return;
  float b0 = 0.f, b1 = 0.f;
  for (int s = 0; s < BN_FS; ++s) {
    b0 += s0[s * BN_FC + cl];
    b1 += s1[s * BN_FC + cl];
  }
  if (mode == 0) {
    mean[c] = b0 / (float)M;
  } else if (mode == 1) {
    const float var = b0 / (float)M;
    rstd[c] = rsqrtf(var + eps);
    if (rmean) {
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean[c];
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
    }
    if (nbt && c == 0) *nbt += 1;
  } else {
    db[c] = b0;
    dw[c] = b1;
  }
}

// Combine per-tile (n_t, mean_t, M2_t) over the ntile row tiles written by a conv epilogue (their row counts n_t in
// `cnt`: 128-row tiles for the generic / 256-row kernels, whole-output-row tiles for the nine-tap forward) with Chan's
// formula, in a fixed order: mean = Σ n_t·mean_t / M,  M2 = Σ M2_t + n_t·(mean_t − mean)².  Then rstd and the
// running statistics as bn_cl_final.  Statistics buffer: [2][ntile][C] tile (mean, M2) | [2][ngroup][C] group
// partials | [ntile] tile counts | [ngroup] group counts (ngroup = ⌈ntile / BN_TG⌉).
// Level 1: one thread per (group of BN_TG tiles, channel) merges its tiles sequentially (Chan's update) into the
// group's (mean, M2); channel 0's thread also writes the group's row count.  The group's loads are issued up front
// (clamped tile index, count 0 past the end) so the sequential merge is not a chain of dependent load latencies.
constexpr int BN_TG = 16;   // tiles per level-1 group: short sequential chains, enough threads (64 measured 35 us/call)
__global__ __launch_bounds__(256) void bn_tile_group(int C, int ntile, const float* __restrict__ ts,
                                                     const float* __restrict__ cnt, float* __restrict__ out,
                                                     float* __restrict__ gcnt) {
  const int ngroup = (ntile + BN_TG - 1) / BN_TG;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)ngroup * C) return;
  const int g = (int)(i / C), c = (int)(i % C);
  float nv[BN_TG], mv[BN_TG], qv[BN_TG];
#pragma unroll
  for (int j = 0; j < BN_TG; ++j) {
    const int t = min(g * BN_TG + j, ntile - 1);
    nv[j] = g * BN_TG + j < ntile ? cnt[t] : 0.f;
    mv[j] = ts[(long)t * C + c];
    qv[j] = ts[((long)ntile + t) * C + c];
  }
  float n = 0.f, mu = 0.f, m2 = 0.f;
#pragma unroll
  for (int j = 0; j < BN_TG; ++j) {
    const float nt = nv[j];
    if (nt <= 0.f) continue;
    const float d = mv[j] - mu, n2 = n + nt;
    mu = fmaf(d, nt / n2, mu);
    m2 += qv[j] + d * d * (n * nt / n2);
    n = n2;
  }
  out[(long)g * C + c] = mu;
  out[((long)ngroup + g) * C + c] = m2;
  if (c == 0) gcnt[g] = n;
}

// Level 2 over the groups (their row counts in gcnt): BN_GC channels per block, BN_GS group slots, each slot with
// BN_FU independent partial sums (fixed-order combine).
constexpr int BN_GC = 4, BN_GS = 256 / BN_GC;
__global__ __launch_bounds__(256) void bn_tile_final(long M, int C, int ngroup, const float* __restrict__ ts,
                                                     const float* __restrict__ gcnt, float* __restrict__ mean,
                                                     float* __restrict__ rstd, float* __restrict__ rmean,
                                                     float* __restrict__ rvar, long long* __restrict__ nbt,
                                                     float momentum, float eps) {
  __shared__ float sh[256];
  __shared__ float smu[BN_GC];
  const int tid = threadIdx.x, cl = tid % BN_GC, slot = tid / BN_GC;
  const int c = blockIdx.x * BN_GC + cl;
  // pass 1: Σ n_g·mean_g;  pass 2: Σ M2_g + n_g·(mean_g − mean)²
  auto sweep = [&](bool second, float mu) {
    float a[BN_FU] = {};
    if (c < C) {
      int t = slot;
      for (; t + (BN_FU - 1) * BN_GS < ngroup; t += BN_FU * BN_GS) {
#pragma unroll
        for (int u = 0; u < BN_FU; ++u) {
          const int tt = t + u * BN_GS;
          const float m = ts[(long)tt * C + c], n = gcnt[tt];
          if (second) {
            const float d = m - mu;
            a[u] += ts[((long)ngroup + tt) * C + c] + n * d * d;
          } else {
            a[u] = fmaf(n, m, a[u]);
          }
        }
      }
      for (; t < ngroup; t += BN_GS) {
        const float m = ts[(long)t * C + c], n = gcnt[t];
        if (second) {
          const float d = m - mu;
          a[0] += ts[((long)ngroup + t) * C + c] + n * d * d;
        } else {
          a[0] = fmaf(n, m, a[0]);
        }
      }
    }
    return (a[0] + a[1]) + (a[2] + a[3]);
  };
  sh[tid] = sweep(false, 0.f);
  __syncthreads();
  if (slot == 0) {
    float b = 0.f;
    for (int k = 0; k < BN_GS; ++k) b += sh[k * BN_GC + cl];
    smu[cl] = b / (float)M;
  }
  __syncthreads();
  const float mu = smu[cl];
  const float q = sweep(true, mu);
  __syncthreads();
  sh[tid] = q;
  __syncthreads();
  if (slot || c >= C) return;
  float m2 = 0.f;
  for (int k = 0; k < BN_GS; ++k) m2 += sh[k * BN_GC + cl];
  const float var = m2 / (float)M;
  mean[c] = mu;
  rstd[c] = rsqrtf(var + eps);
  if (rmean) {
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
  }
  if (nbt && c == 0) *nbt += 1;
}

// Row counts of the tile statistics: where a conv epilogue writes n_t (after the tile and group partials)
__device__ __forceinline__ float* tile_counts(float* ts, int ntile, int C) {
  return ts + 2L * (ntile + (ntile + BN_TG - 1) / BN_TG) * C;
}

// Per-column BatchNorm statistics (mean, Σ(v − mean)²) of the bf16-rounded values of a conv tile's fp32 LDS staging
// image, by ALL NT threads of the block: ncols (dividing NT) columns, P = NT / ncols row partitions per column (rows
// p, p + P, …), partials combined in a fixed order through `scr` (2·NT floats of LDS outside the image).  One thread
// per column walking up to 256 rows twice left each tile a long single-wave tail (the other waves idle, the CU's
// workgroup slot held).  Every thread of the block must call it (two barriers).  val(c, r): image value of column c,
// row r; nrows(c): valid rows of column c (≤ 0: none); out(c, mean, m2) runs on one thread per column.
template <int NT, typename V, typename NR, typename OUT>
__device__ __forceinline__ void tile_col_stats(int ncols, float* scr, int tid, V val, NR nrows, OUT out) {
  const int P = NT / ncols, c = tid % ncols, p = tid / ncols;
  const int rows = nrows(c);
  float s = 0.f;
  for (int r = p; r < rows; r += P) s += (float)(bf16)val(c, r);
  scr[tid] = s;
  __syncthreads();
  float mu = 0.f;
  for (int q = 0; q < P; ++q) mu += scr[q * ncols + c];
  mu = rows > 0 ? mu / (float)rows : 0.f;
  float m2 = 0.f;
  for (int r = p; r < rows; r += P) {
    const float d = (float)(bf16)val(c, r) - mu;
    m2 = fmaf(d, d, m2);
  }
  scr[NT + tid] = m2;
  __syncthreads();
  if (p == 0 && rows > 0) {
    float t = 0.f;
    for (int q = 0; q < P; ++q) t += scr[NT + q * ncols + c];
    out(c, mu, t);
  }
}

__global__ void bn_cl_eval_stats(int C, const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                 float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) { mean[c] = rmean[c]; rstd[c] = rsqrtf(rvar[c] + eps); }
}

// y = act((x − mean)·rstd·w + b + res), act = identity / ReLU (relu 1) / ReLU6 (relu 2), 8 channels per thread.
// HOIST (C/8 divides 256, so a thread's channels never change along the grid-stride loop): the per-channel
// constants are loaded once per thread instead of once per vector (8 of the 10 loads of an iteration).
template <typename T, bool HOIST>
__global__ __launch_bounds__(256) void bn_cl_apply(unsigned nvec, int C, const T* __restrict__ x,
                                                   const T* __restrict__ res, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* __restrict__ w,
                                                   const float* __restrict__ b, int relu, T* __restrict__ y) {
  const unsigned cv = C / 8;
  float mu[8], rs[8], ww[8], bb[8];
  // per-channel constants as explicit 16-B loads (c0 % 8 == 0; the per-element form lost its vectorisation
  // once the activation became a two-way choice: 34 vs 10 loads per 8 channels, 4x slower)
  auto consts = [&](unsigned i) {
    const int c0 = (int)(i % cv) * 8;
    Vec8<float>::load(mean + c0, mu);
    Vec8<float>::load(rstd + c0, rs);
    Vec8<float>::load(w + c0, ww);
    Vec8<float>::load(b + c0, bb);
  };
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (HOIST) consts(i0);
  const float lo = relu ? 0.f : -INFINITY, hi = relu == 2 ? 6.f : INFINITY;
  for (unsigned i = i0; i < nvec; i += gridDim.x * blockDim.x) {
    const long off = (long)i * 8;
    float v[8], rv[8];
    Vec8<T>::load(x + off, v);
    if (res) Vec8<T>::load(res + off, rv);
    if (!HOIST) consts(i);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = fmaf((v[j] - mu[j]) * rs[j], ww[j], bb[j]);
      if (res) v[j] += rv[j];
      v[j] = fminf(fmaxf(v[j], lo), hi);
    }
    Vec8<T>::store(y + off, v);
  }
}

// g = dy·act'(y);  dres = g (optional);  dx = w·rstd·(g − Σg/M − x̂·Σgx̂/M) (training) or w·rstd·g (eval).
// relu | BN_ZMASK: act'(y) recomputed from x (no residual; see bn_cl_partial), y not read.  HOIST: as bn_cl_apply.
template <typename T, bool HOIST>
__global__ __launch_bounds__(256) void bn_cl_bwd_apply(unsigned nvec, int M, int C, const T* __restrict__ x,
                                                       const T* __restrict__ y, const T* __restrict__ dy,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       const float* __restrict__ dw, const float* __restrict__ db,
                                                       int training, int relu, T* __restrict__ dx,
                                                       T* __restrict__ dres) {
  const float inv = 1.f / (float)M;
  const unsigned cv = C / 8;
  const bool zm = relu & BN_ZMASK, ry = relu && !zm, needx = training || zm;
  float rs[8], ww[8], mu[8], sw[8], sb[8], bb[8];
  // per-channel constants as explicit 16-B loads (c0 % 8 == 0): per element they compiled to 40 scalar loads
  auto consts = [&](unsigned i) {
    const int c0 = (int)(i % cv) * 8;
    Vec8<float>::load(rstd + c0, rs);
    Vec8<float>::load(w + c0, ww);
    if (needx) Vec8<float>::load(mean + c0, mu);
    if (training) {
      Vec8<float>::load(dw + c0, sw);
      Vec8<float>::load(db + c0, sb);
    }
    if (zm) Vec8<float>::load(b + c0, bb);
  };
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (HOIST) consts(i0);
  for (unsigned i = i0; i < nvec; i += gridDim.x * blockDim.x) {
    const long off = (long)i * 8;
    float gv[8], yv[8], xv[8], out[8];
    Vec8<T>::load(dy + off, gv);
    if (ry) Vec8<T>::load(y + off, yv);
    if (needx) Vec8<T>::load(x + off, xv);
    if (!HOIST) consts(i);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (zm ? !bn_act_on<T>(fmaf((xv[j] - mu[j]) * rs[j], ww[j], bb[j]), relu) : ry && !bn_y_on(yv[j], relu))
        gv[j] = 0.f;
      if (training) {
        const float xh = (xv[j] - mu[j]) * rs[j];
        out[j] = ww[j] * rs[j] * (gv[j] - sb[j] * inv - xh * sw[j] * inv);
      } else {
        out[j] = ww[j] * rs[j] * gv[j];
      }
    }
    if (dres) Vec8<T>::store(dres + off, gv);
    Vec8<T>::store(dx + off, out);
  }
}

// Global average pool over the S positions of each clip: [N, S, C] → fp32 [N, C]; backward broadcasts dout/S.
template <typename T>
__global__ __launch_bounds__(256) void avgpool_cl_fwd(int N, long S, int C, const T* __restrict__ x,
                                                      float* __restrict__ out) {
  __shared__ float sh[256];
  const int n = blockIdx.y, tid = threadIdx.x;
  const int CB = C < 256 ? C : 256, RPI = 256 / CB, slot = tid / CB, cc = tid % CB;
  for (int c0 = blockIdx.x * CB; c0 < C; c0 += gridDim.x * CB) {
    float a = 0.f;
    if (slot < RPI && c0 + cc < C)      // (C not a multiple of CB / CB not dividing 256: spare threads add 0)
      for (long s = slot; s < S; s += RPI) a += to_f<T>(x[((long)n * S + s) * C + c0 + cc]);
    sh[tid] = a;
    __syncthreads();
    if (slot == 0 && c0 + cc < C) {
      float b = 0.f;
      for (int k = 0; k < RPI; ++k) b += sh[k * CB + cc];
      out[(long)n * C + c0 + cc] = b / (float)S;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(256) void avgpool_cl_bwd(long total, long S, int C, const float* __restrict__ dout,
                                                      T* __restrict__ dx) {
  const float inv = 1.f / (float)S;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long n = i / C / S;
    dx[i] = from_f<T>(dout[n * C + c] * inv);
  }
}

// (B, T, C, H, W) fp32 video → (B, T, H, W, C) compute dtype.
template <typename T>
__global__ __launch_bounds__(256) void video_ndhwc_kernel(long total, int C, long HW, const float* __restrict__ v,
                                                          T* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long p = i / C;          // (b·T + t)·HW + hw
    const long bt = p / HW, hw = p - bt * HW;
    out[i] = from_f<T>(v[(bt * C + c) * HW + hw]);
  }
}

// ---- implicit-GEMM conv3d on MFMA (bf16, C % 64 == 0: a 64-wide K-tile never crosses a tap) ----------------------
// Same tile machinery as gemm_bf16.hip's 128² kernel (128x128x64 tile, 4 waves of 64x64 = 4x4
// mfma_f32_16x16x32_bf16, XOR-swizzled LDS images, register-staged double buffer, one barrier per K-tile), with the
// column matrix never materialised: the im2col gather happens in the operand loads.
//   forward  z[m, co]  = Σ_k col(m, k)·W[co, k]         A = col (gathered, K-contiguous), B = W [Cout][K]
//   wgrad    dW[co, k] = Σ_m dz[m, co]·col(m, k)       A = dz (row-contraction), B = col (gathered, row-contraction)
namespace ig {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256, EPI_LD = BN + 4;
__device__ __forceinline__ int kc_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int mc_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int mc_off(int k, int chunk) { return k * 256 + ((chunk ^ mc_swz(k)) << 4); }

template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* lds, int r0, int kk, int lane) {
  if (KC) {
    return *(const bf16x8*)(lds + kc_off(r0 + (lane & 15), kk * 4 + (lane >> 4)));
  } else {
    const int gq = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (r0 >> 3) + (p >> 1);
    const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(short4_t, lds + mc_off(kk * 32 + 8 * gq + q, chunk) + (p & 1) * 8));
    const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(short4_t, lds + mc_off(kk * 32 + 8 * gq + 4 + q, chunk) + (p & 1) * 8));
    short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Input element offset of output position m for tap (it, ih, iw), or -1 when it falls in the zero padding.
__device__ __forceinline__ long tap_src(const Geom& g, int n, int t0, int h0, int w0, int it, int ih, int iw) {
  const int ti = t0 + it, hi = h0 + ih, wi = w0 + iw;
  if (ti < 0 || ti >= g.T || hi < 0 || hi >= g.H || wi < 0 || wi >= g.W) return -1;
  return ((((long)n * g.T + ti) * g.H + hi) * g.W + wi) * g.C;
}
__device__ __forceinline__ void out_pos(const Geom& g, int m, int& n, int& t0, int& h0, int& w0) {
  int r = m;
  const int wo = r % g.Wo; r /= g.Wo;
  const int ho = r % g.Ho; r /= g.Ho;
  const int to = r % g.To;
  n = r / g.To;
  t0 = to * g.st - g.pt; h0 = ho * g.sh - g.ph; w0 = wo * g.sw - g.pw;
}

// JN = 16-column blocks per wave: 4 (128-wide tile) or 2 (64-wide tile, for Cout = 64 convs)
template <bool AKC, bool BKC, int JN>
__device__ __forceinline__ void mma_tile(const char* As, const char* Bs, int wr, int wc, int lane,
                                         floatx4 (&acc)[4][JN]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 af[4], bfr[JN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag<AKC>(As, wr * 64 + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < JN; ++j) bfr[j] = frag<BKC>(Bs, wc * JN * 16 + j * 16, kk, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
}

// Stage the fp32 accumulators through LDS and emit rows [bm, min(bm+128, M)) x cols [bn, min(bn+128, N)) with
// 8-column vectors (N % 8 == 0).
template <typename OutT, int JN>
__device__ __forceinline__ void store_tile(char* smem, const floatx4 (&acc)[4][JN], int wr, int wc, int lane, int tid,
                                           int bm, int bn, int M, int N, OutT* __restrict__ C, long ldc,
                                           const OutT* __restrict__ res = nullptr) {
  constexpr int TPR = JN * 4;                      // threads per output row (8 columns each)
  constexpr int LD = JN * 32 + 4;                  // padded fp32 staging row
  float* T = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wr * 64 + i * 16 + 4 * (lane >> 4) + r) * LD + wc * JN * 16 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int cg = (tid % TPR) * 8, n0 = bn + cg;
  if (n0 >= N) return;
  for (int rr = tid / TPR; rr < BM; rr += NT / TPR) {
    const int m = bm + rr;
    if (m >= M) break;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = T[rr * LD + cg + j];
    if (res) {
      float r[8];
      vload<OutT, 8>(res + (long)m * ldc + n0, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    vstore<OutT, 8>(C + (long)m * ldc + n0, v);
  }
}
}  // namespace ig

// LDS: A stages 2 x 16 KiB, B stages 2 x (JN·4 KiB), fp32 staging 128 x (32·JN + 4) — 48 KiB at JN = 2, so three
// workgroups share a CU (vs two at JN = 4).
template <int JN> struct FwdLds {
  static constexpr int B0 = 32768, BSTAGE = JN * 4096;
  static constexpr int OPS = B0 + 2 * BSTAGE, EPI = 128 * (JN * 32 + 4) * 4;
  static constexpr int BYTES = OPS > EPI + 2048 ? OPS : EPI + 2048;   // + tile_col_stats scratch past the image
};

template <int JN, bool BUF>
__global__ __launch_bounds__(256, JN == 2 ? 3 : 2) void conv3d_fwd_igemm(Geom g, int M, int Cout, const bf16* __restrict__ x,
                                                           const bf16* __restrict__ Wt, const bf16* __restrict__ res,
                                                           bf16* __restrict__ z, float* __restrict__ tstats, int kps,
                                                           float* __restrict__ part) {
  using namespace ig;
  using Lds = FwdLds<JN>;
  __shared__ __attribute__((aligned(16))) char smem[Lds::BYTES];
  constexpr int TN = JN * 32, NB = TN / 32;        // tile width (Cout) and B-row loads per thread
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  const int tiles_n = (Cout + TN - 1) / TN, ntile = ((M + BM - 1) / BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  const int bm = (bid / tiles_n) * BM, bn = (bid % tiles_n) * TN;
  // this thread's four A rows (row = it*32 + tid/8) are fixed for the whole K loop: decompose them once
  int an[4], at[4], ah[4], aw[4];
  bool aok[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int m = bm + it * 32 + (tid >> 3);
    aok[it] = m < M;
    out_pos(g, aok[it] ? m : 0, an[it], at[it], ah[it], aw[it]);
  }
  const int kk8 = (tid & 7) * 8;
  uint4_t ra[4], rb[4];
  // BUF: operands through buffer resources with 32-bit byte offsets (x and the weights under 2 GiB); padding and
  // out-of-range rows / columns load from offset 2^31, past the resource, which reads zeros (as conv3d_fwd_rows3).
  // Otherwise 64-bit addresses, the padding zeroed at the LDS store.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);
  unsigned am = 0, bmk = 0;   // !BUF: in-range bits of ra / rb
  auto load = [&](int k0) {
    const int tap = k0 / g.C, c0 = k0 - tap * g.C + kk8;
    const int iw = tap % g.kw, ih = (tap / g.kw) % g.kh, itp = tap / (g.kw * g.kh);
    am = bmk = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const long off = aok[it] ? tap_src(g, an[it], at[it], ah[it], aw[it], itp, ih, iw) : -1;
      if constexpr (BUF) {
        const unsigned bo = off >= 0 ? (unsigned)((off + c0) * 2) : 0x80000000u;
        ra[it] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, bo, 0, 0));
      } else {
        ra[it] = *(const uint4_t*)(x + (off >= 0 ? off + c0 : 0));
        am |= (unsigned)(off >= 0) << it;
      }
    }
#pragma unroll
    for (int it = 0; it < NB; ++it) {
      const int co = bn + it * 32 + (tid >> 3);
      if constexpr (BUF) {
        const unsigned bo = co < Cout ? (unsigned)((co * g.Kp + k0 + kk8) * 2) : 0x80000000u;
        rb[it] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(wrs, bo, 0, 0));
      } else {
        rb[it] = *(const uint4_t*)(Wt + (long)(co < Cout ? co : 0) * g.Kp + k0 + kk8);
        bmk |= (unsigned)(co < Cout) << it;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int off = kc_off(it * 32 + (tid >> 3), tid & 7);
      *(uint4_t*)(smem + 16384 * buf + off) = BUF ? ra[it] : zero_unless((am >> it) & 1, ra[it]);
      if (it < NB)
        *(uint4_t*)(smem + Lds::B0 + Lds::BSTAGE * buf + off) = BUF ? rb[it] : zero_unless((bmk >> it) & 1, rb[it]);
    }
  };
  floatx4 acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // K-steps [kb, ke): all of them, or split blockIdx.y's share (part: its fp32 partial tile, no statistics)
  const int nk = g.K / BK, kb = blockIdx.y * kps, ke = min(nk, kb + kps);
  load(kb * BK);
  store(0);
  __syncthreads();
  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) & 1;
    const bool more = kt + 1 < ke;
    if (more) load((kt + 1) * BK);
    if (CMHAR_IGEMM_PRIO) __builtin_amdgcn_s_setprio(1);
    mma_tile<true, true, JN>(smem + 16384 * cur, smem + Lds::B0 + Lds::BSTAGE * cur, wr, wc, lane, acc);
    if (CMHAR_IGEMM_PRIO) __builtin_amdgcn_s_setprio(0);
    if (more) store(cur ^ 1);
    __syncthreads();
  }
  if (part) {
    store_tile<float, JN>(smem, acc, wr, wc, lane, tid, bm, bn, M, Cout, part + (long)blockIdx.y * M * Cout, Cout);
    return;
  }
  store_tile<bf16, JN>(smem, acc, wr, wc, lane, tid, bm, bn, M, Cout, z, Cout, res);
  if (tstats) {
    // BatchNorm statistics of this tile's (bf16-rounded) outputs, per column: tile mean and Σ(v − mean)² over its
    // valid rows, from the fp32 staging image still in LDS (combined across tiles by bn_tile_final, Chan's formula)
    const float* T = (const float*)smem;
    const int rows = min(BM, M - bm), tm = bm / BM, ntm = gridDim.x / ((Cout + TN - 1) / TN);
    tile_col_stats<NT>(TN, (float*)(smem + Lds::EPI), tid, [&](int c, int r) { return T[r * (TN + 4) + c]; },
                       [&](int) { return rows; }, [&](int c, float mu, float m2) {
                         if (bn + c < Cout) {
                           tstats[(long)tm * Cout + bn + c] = mu;
                           tstats[((long)ntm + tm) * Cout + bn + c] = m2;
                         }
                       });
    if (tid == 0 && bn == 0) tile_counts(tstats, ntm, Cout)[tm] = (float)rows;
  }
}

// dW partial over output rows [z·mlen, min(M, (z+1)·mlen)) into ws slab z (fp32 [Cout][K]).
__global__ __launch_bounds__(256, 2) void conv3d_wgrad_igemm(Geom g, int M, int Cout, int mlen,
                                                             const bf16* __restrict__ x, const bf16* __restrict__ dz,
                                                             float* __restrict__ out) {
  using namespace ig;
  __shared__ __attribute__((aligned(16))) char smem[BM * EPI_LD * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  const int tiles_n = (g.K + BN - 1) / BN, ntile = ((Cout + BM - 1) / BM) * tiles_n;
  const int rl = xcd_remap(blockIdx.x + ntile * blockIdx.y, ntile * gridDim.y);
  const int bid = rl % ntile, split = rl / ntile;
  const int bm = (bid / tiles_n) * BM, bn = (bid % tiles_n) * BN;   // bm: Cout rows, bn: K columns
  const int mbeg = split * mlen, mend = min(M, mbeg + mlen);
  // this thread's B columns (8 consecutive k of one tap) are fixed: decompose the tap once
  const int kq = (tid & 15) * 8;                  // non-K-contiguous image: 16 x 8 columns per row
  const int kcol = bn + kq;
  const bool kok = kcol < g.K;
  const int tap = kok ? kcol / g.C : 0, cc = kok ? kcol - tap * g.C : 0;
  const int iw = tap % g.kw, ih = (tap / g.kw) % g.kh, itp = tap / (g.kw * g.kh);
  const int co = bm + kq;
  const bool cok = co < Cout;
  // Two register sets: tile t+2's gather is issued while tile t is multiplied and tile t+1 (loaded one full
  // iteration earlier) is written to LDS, so each scattered load has two MFMA phases to land.
  uint4_t ra0[4], rb0[4], ra1[4], rb1[4];
  auto load = [&](int m0, uint4_t (&ra)[4], uint4_t (&rb)[4]) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int m = m0 + it * 16 + (tid >> 4);
      const bool mok = m < mend;
      const uint4_t a = *(const uint4_t*)(dz + (long)(mok ? m : 0) * Cout + (cok ? co : 0));
      ra[it] = mok && cok ? a : uint4_t{0u, 0u, 0u, 0u};
      long off = -1;
      if (mok && kok) {
        int n, t0, h0, w0;
        out_pos(g, m, n, t0, h0, w0);
        off = tap_src(g, n, t0, h0, w0, itp, ih, iw);
      }
      const uint4_t b = *(const uint4_t*)(x + (off >= 0 ? off + cc : 0));
      rb[it] = off >= 0 ? b : uint4_t{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf, const uint4_t (&ra)[4], const uint4_t (&rb)[4]) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int off = mc_off(it * 16 + (tid >> 4), tid & 15);
      *(uint4_t*)(smem + 16384 * buf + off) = ra[it];
      *(uint4_t*)(smem + 32768 + 16384 * buf + off) = rb[it];
    }
  };
  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = mend > mbeg ? (mend - mbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load(mbeg, ra0, rb0);
    store(0, ra0, rb0);
    if (nk > 1) load(mbeg + BK, ra1, rb1);
  }
  __syncthreads();
  // tile kt lives in LDS buffer kt&1 and was loaded into register set kt&1
  auto step = [&](int kt, uint4_t (&rac)[4], uint4_t (&rbc)[4], uint4_t (&ran)[4], uint4_t (&rbn)[4]) {
    if (kt + 2 < nk) load(mbeg + (kt + 2) * BK, rac, rbc);
    mma_tile<false, false, 4>(smem + 16384 * (kt & 1), smem + 32768 + 16384 * (kt & 1), wr, wc, lane, acc);
    if (kt + 1 < nk) store((kt + 1) & 1, ran, rbn);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, ra0, rb0, ra1, rb1);
    if (kt + 1 < nk) step(kt + 1, ra1, rb1, ra0, rb0);
  }
  store_tile<float, 4>(smem, acc, wr, wc, lane, tid, bm, bn, Cout, g.K, out + (long)split * Cout * g.K, g.K);
}

// ---- weight gradient of the k x k x 3 convolutions from input row slabs ------------------------------------------
// dW[co, (it, ih, iw), c] = Σ_m dz[m, co] · x[in(m, it, ih) + iw, c].  The generic kernel above gathers a fresh
// input row for every (m, tap) of its 128-column tile, so the input is read once per tap (27× per conv).  Here a
// workgroup owns one (it, ih) tap pair, one 64-channel slice and all three kw taps (192 dW columns), and walks the
// output rows in chunks of R = ⌊64 / Wo⌋ whole rows: per chunk it stages the chunk's dz rows (a contiguous
// [R·Wo][Cout-tile] block) and, per output row, the ONE input row segment its three kw taps read (Ls = (Wo−1)·sw + 3
// positions) — the kw taps are then row shifts of the same LDS slab.  The input is read kt·kh = 9 times instead of
// 27, dz 9 times per Cout tile instead of once per 128-column tile, and no MFMA work is spent on padding columns.
namespace wr {
constexpr int SLOTS = 64, MAXQ = 136, RS = 144;   // RS: LDS row stride in bytes (128 + 16 pad)
// [row][64 bf16] images with 144-B rows: every fragment address is a per-lane base plus a compile-time offset (no
// per-(tap, column block) address registers), and the 16 rows of one transposed read (rows 8g + q of a half-wave)
// start 36 banks apart: at most 2 lanes of a 32-lane half per bank for unit and stride-2 row steps
// (cdna_hip_programming.md: ds_read_b64_tr_b16 banks are (a/4) % 64 per 32-lane half).
// 16x16x32 operand fragment: 4 bf16 of rows lo and hi (lo = k 8g + q, hi = k 8g + 4 + q of this lane) at column
// block offset; `lo`/`hi` are byte addresses of this lane's rows + its chunk / half offset
__device__ __forceinline__ bf16x8 frag_at(const char* lo, const char* hi) {
  const short4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lo));
  const short4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, hi));
  short8_t v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}
}  // namespace wr

// COT = Cout tile (64 or 128): dz image COT/64 sub-images of [64 slots][64].  G = kh taps per workgroup (1, or 3:
// the whole kh column for one it — the dz chunk then feeds 576 dW columns); SQ = slab rows per tap; NW waves split
// the G·12 16-column blocks evenly, each covering every Cout row of the tile.  Operands are register-staged one chunk
// ahead (an LDS-DMA ring 2–3 chunks ahead at one workgroup per CU measured 1.2–2.2× slower: its per-piece issue
// cost and the single wave per SIMD outweigh the deeper prefetch).  Every division of the gather is done once per
// thread (the chunk-invariant slot → row / position map) or once per chunk (the chunk's first output row).
template <int COT, int G, int SQ, int NW>
__global__ __launch_bounds__(64 * NW, 2) void conv3d_wgrad_rows(Geom g, int Cout, int R, int Ls, int rows_total,
                                                               int chunks_per_split, const bf16* __restrict__ x,
                                                               const bf16* __restrict__ dz, float* __restrict__ out) {
  using namespace wr;
  constexpr int NT = 64 * NW, NCB = COT / 16, NJ = 12 * G / NW, DZ_SUB = SLOTS * RS, DZ_BYTES = (COT / 64) * DZ_SUB;
  static_assert(NJ * NW == 12 * G, "column blocks must split evenly over the waves");
  constexpr int SLAB_BYTES = G * SQ * RS, DZ_N = SLOTS * COT / 8, SL_N = G * SQ * 8;
  constexpr int DZ_PER = (DZ_N + NT - 1) / NT, SL_PER = (SL_N + NT - 1) / NT;
  constexpr int BUF = DZ_BYTES + SLAB_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nct = g.C / 64, ncot = Cout / COT, ngrp = g.kt * (g.kh / G), ntile = ngrp * nct * ncot;
  const int lin = xcd_remap(blockIdx.x + ntile * blockIdx.y, ntile * gridDim.y);   // one split's tiles per XCD
  const int split = lin / ntile;
  int tl = lin % ntile;
  const int cot = tl % ncot; tl /= ncot;
  const int ct = tl % nct; tl /= nct;
  const int ih0 = (tl % (g.kh / G)) * G, it = tl / (g.kh / G);
  const int nchunk = (rows_total + R - 1) / R;
  const int c_beg = split * chunks_per_split, c_end = min(nchunk, c_beg + chunks_per_split);
  const int M = rows_total * g.Wo, used = R * g.Wo, nq = R * Ls;
  // chunk-invariant part of this thread's slab loads: output row r within the chunk (-1: none), input position
  // wi, input row offset hi − ho·sh (the tap), column
  int sr[SL_PER], swi[SL_PER], sdh[SL_PER];
#pragma unroll
  for (int i = 0; i < SL_PER; ++i) {
    const int e = i * NT + tid, qq = e >> 3;
    const int gi = qq / SQ, q2 = qq - gi * SQ;
    sr[i] = -1; swi[i] = 0; sdh[i] = 0;
    if (e < SL_N && gi < G && q2 < nq) {
      const int r = q2 / Ls;
      sr[i] = r;
      swi[i] = q2 - r * Ls - g.pw;
      sdh[i] = ih0 + gi - g.ph;
    }
  }
  // this lane's fragment rows: dz slot rows k = 32kk + 8g + 4hh + q; slab rows of tap iw = 0 for those slots (slots
  // past R·Wo read row 0: their dz is zero).  Byte offsets include the lane's chunk (p>>1) and half (p&1).
  const int gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int lane_col = (p >> 1) * 16 + (p & 1) * 8;
  int sl_off[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int k = 32 * kk + 8 * gq + 4 * hh + q;
      sl_off[kk][hh] = (k < used ? (k / g.Wo) * Ls + (k % g.Wo) * g.sw : 0) * RS + lane_col;
    }
  const int dz_off = (8 * gq + q) * RS + lane_col;
  // operands through buffer resources with 32-bit byte offsets (the plan keeps x and dz within 1 GiB); padding and
  // out-of-range slots load from offset 2^31, past the resource, which reads zeros (as conv3d_fwd_rows3)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t dzr = __builtin_amdgcn_make_buffer_rsrc((void*)dz, (short)0, (int)min((long)M * Cout * 2, 0x7fffffffL),
                                                                        0x00020000);
  uint4_t rdz[DZ_PER], rsl[SL_PER];
  auto load = [&](int c) {
    const int rho0 = c * R;
    const int m0 = rho0 * g.Wo;
    const int ho0 = rho0 % g.Ho, tn0 = rho0 / g.Ho, to0 = tn0 % g.To, n0 = tn0 / g.To;
#pragma unroll
    for (int i = 0; i < DZ_PER; ++i) {
      const int e = i * NT + tid, j = e / (COT / 8), ch = e % (COT / 8);
      const bool ok = e < DZ_N && j < used && m0 + j < M;
      const unsigned off = ok ? (unsigned)(((m0 + j) * Cout + cot * COT + ch * 8) * 2) : 0x80000000u;
      rdz[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(dzr, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      unsigned off = 0x80000000u;
      if (sr[i] >= 0 && rho0 + sr[i] < rows_total) {
        int ho = ho0 + sr[i], to = to0, n = n0;
        while (ho >= g.Ho) {          // at most R / Ho + 1 wraps
          ho -= g.Ho;
          if (++to == g.To) { to = 0; ++n; }
        }
        const int ti = to * g.st - g.pt + it, hi = ho * g.sh + sdh[i], wi = swi[i];
        if (ti >= 0 && ti < g.T && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
          off = (unsigned)(((((n * g.T + ti) * g.H + hi) * g.W + wi) * g.C + ct * 64 + ((i * NT + tid) & 7) * 8) * 2);
      }
      rsl[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store = [&](int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < DZ_PER; ++i) {
      const int e = i * NT + tid, j = e / (COT / 8), ch = e % (COT / 8);
      if (e < DZ_N) *(uint4_t*)(base + (ch >> 3) * DZ_SUB + j * RS + (ch & 7) * 16) = rdz[i];
    }
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      const int e = i * NT + tid, qq = e >> 3, ch = e & 7;
      if (e < SL_N) *(uint4_t*)(base + DZ_BYTES + qq * RS + ch * 16) = rsl[i];
    }
  };
  floatx4 acc[NCB][NJ];
#pragma unroll
  for (int i = 0; i < NCB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (c_beg < c_end) {
    load(c_beg);
    store(0);
  }
  __syncthreads();
  for (int c = c_beg; c < c_end; ++c) {
    const int cur = (c - c_beg) & 1;
    const bool more = c + 1 < c_end;
    if (more) load(c + 1);
    const char* dzs = smem + cur * BUF;
    const char* sls = dzs + DZ_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[NCB];
#pragma unroll
      for (int i = 0; i < NCB; ++i) {
        const char* a = dzs + (i >> 2) * DZ_SUB + dz_off + 32 * kk * RS + (i & 3) * 32;
        af[i] = frag_at(a, a + 4 * RS);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cb = NJ * wave + j, gi = cb / 12, iw = (cb % 12) >> 2;
        const int cofs = (gi * SQ + iw) * RS + (cb & 3) * 32;
        const bf16x8 bf = frag_at(sls + sl_off[kk][0] + cofs, sls + sl_off[kk][1] + cofs);
#pragma unroll
        for (int i = 0; i < NCB; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][j], 0, 0, 0);
      }
    }
    if (more) store(cur ^ 1);
    __syncthreads();
  }
  // partial dW of this split: rows co = cot·COT + 16i + 4(lane>>4) + r, columns k = ((it·kh + ih)·kw + iw)·C +
  // ct·64 + 16(cb&3) + (lane&15)
  float* o = out + (long)split * Cout * g.K;
#pragma unroll
  for (int i = 0; i < NCB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cb = NJ * wave + j, gi = cb / 12, iw = (cb % 12) >> 2;
      const long col = ((long)(it * g.kh + ih0 + gi) * g.kw + iw) * g.C + ct * 64 + (cb & 3) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cot * COT + 16 * i + 4 * (lane >> 4) + r;
        o[(long)co * g.K + col] = acc[i][j][r];
      }
    }
}

// Stride-1 H/W variant: a workgroup owns one it, one 64-channel slice of the input, one 64-wide Cout slice and ALL
// nine (ih, iw) taps (576 dW columns, 12 waves x 3 column blocks), and a chunk is up to R <= ⌊256 / Wo⌋ consecutive
// output rows of one frame (R balanced over the frame's rows):
// output row r and tap ih read input row r + ih, so the chunk's R + 2 input row segments serve all 3·R (row, ih)
// pairs (the one-tap-row kernel stages 3·R) and each staged dz row feeds 576 columns instead of 192 — 2.3x the
// MFMA work per staged byte for R3D-18 layer 1 (R = 4).
namespace wr3 {
constexpr int SLOTS = 256, SQ = 352, RS = 144;
constexpr int DZB = SLOTS * RS, DZ_N = SLOTS * 8;
// CS = input channels per workgroup: 64 (one 12-wave workgroup per CU, 36 column blocks) or 32 (CMHAR_WGRAD3_CS=32:
// two 6-wave workgroups per CU, 18 column blocks each, 80-B slab rows — each stages the dz chunk itself, and the two
// run out of phase, one's LDS stores and barriers beside the other's MFMAs).  Round 6 (168 VGPRs,
// 65 KB LDS, R3D tests green): layer 1 / 2 / 3 weight gradients 405.7 / 207.5 / 114.3 -> 524.9 / 288.7 / 154.5 us,
// the R3D-18 step 2218 / 2253 -> 2192 / 2167 clips/s — the duplicated dz staging costs more than the overlap wins; 64)
template <int CS> struct C3 {
  static constexpr int NW = CS == 64 ? 12 : 6, NT = 64 * NW, CPT = CS / 16, NCB = 9 * CPT;
  static constexpr int SLC = CS / 8, RSL = CS * 2 + 16;               // 16-B chunks per slab slot, slab row bytes
  static constexpr int SLB = SQ * RSL, SL_N = SQ * SLC;
  static constexpr int DZ_PER = (DZ_N + NT - 1) / NT, SL_PER = (SL_N + NT - 1) / NT;
  static_assert(NCB == 3 * NW, "three column blocks per wave");
};
}  // namespace wr3

template <int CS>
__global__ __launch_bounds__(wr3::C3<CS>::NT, CS == 64 ? 1 : 2) void conv3d_wgrad_rows3(
    Geom g, int Cout, int R, int Ls, int cpf, int nchunk, int chunks_per_split, const bf16* __restrict__ x,
    const bf16* __restrict__ dz, float* __restrict__ out) {
  using namespace wr3;
  typedef C3<CS> Q;
  constexpr int NT = Q::NT, RSL = Q::RSL, SLC = Q::SLC, CPT = Q::CPT, DZ_PER = Q::DZ_PER, SL_PER = Q::SL_PER;
  __shared__ __attribute__((aligned(16))) char smem[DZB + Q::SLB];
  char* const dzs = smem;
  char* const sls = smem + DZB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nct = g.C / CS, ncot = Cout / 64, ntile = g.kt * nct * ncot;
  const int lin = xcd_remap(blockIdx.x + ntile * blockIdx.y, ntile * gridDim.y);
  const int split = lin / ntile;
  int tl = lin % ntile;
  const int cot = tl % ncot; tl /= ncot;
  const int ct = tl % nct;
  const int it = tl / nct;
  const int c_beg = split * chunks_per_split, c_end = min(nchunk, c_beg + chunks_per_split);
  // operands through buffer resources with 32-bit byte offsets (the plan keeps x and dz within 1 GiB); padding and
  // out-of-range slots load from offset 2^31, past the resource, which reads zeros (as conv3d_fwd_rows3)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t dzr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dz, (short)0, (int)min((long)g.N * g.To * g.Ho * g.Wo * Cout * 2, 0x7fffffffL), 0x00020000);
  // chunk-invariant slab slots: input row u of the chunk's slab and the byte offset of the slot's 16 B relative to
  // the slab's first input row (-1 in the W padding)
  int su[SL_PER], sb[SL_PER];
#pragma unroll
  for (int i = 0; i < SL_PER; ++i) {
    const int q = (i * NT + tid) / SLC;
    su[i] = q / Ls;
    const int wi = q - su[i] * Ls - g.pw;
    sb[i] = wi >= 0 && wi < g.W ? ((su[i] * g.W + wi) * g.C + ct * CS + ((i * NT + tid) % SLC) * 8) * 2 : -1;
  }
  // fragment rows of this lane: slot k → (r, wo) → slab row r·Ls + wo (+ ih·Ls + iw per column block); slots past
  // the chunk's rows read row 0 (their dz is zero)
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p = lane & 3;
  const int lane_col = (p >> 1) * 16 + (p & 1) * 8;
  const int used_max = R * g.Wo;
  int sl_off[8][2];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int k = 32 * kk + 8 * gq + 4 * hh + q4;
      sl_off[kk][hh] = (k < used_max ? (k / g.Wo) * Ls + (k % g.Wo) : 0) * RSL + lane_col;
    }
  const int dz_off = (8 * gq + q4) * RS + lane_col;
  uint4_t rdz[DZ_PER], rsl[SL_PER];
  auto load = [&](int c) {
    const int f = c / cpf, ho0 = (c - f * cpf) * R, nr = min(R, g.Ho - ho0);
    const int to = f % g.To, n = f / g.To;
    const int m0 = (f * g.Ho + ho0) * g.Wo;
    const int used = nr * g.Wo;
#pragma unroll
    for (int i = 0; i < DZ_PER; ++i) {
      const int e = i * NT + tid, j = e >> 3, ch = e & 7;
      const unsigned off = e < DZ_N && j < used ? (unsigned)(((m0 + j) * Cout + cot * 64 + ch * 8) * 2) : 0x80000000u;
      rdz[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(dzr, off, 0, 0));
    }
    // slab row u is input row ho0 − ph + u of frame ti: in range for u in [u_lo, u_hi) (none when ti is padding)
    const int ti = to * g.st - g.pt + it;
    const bool tok = ti >= 0 && ti < g.T;
    const int u_lo = tok ? g.ph - ho0 : 0x7fffffff, u_hi = min(g.H + g.ph - ho0, nr + 2);
    const int base = (((n * g.T + ti) * g.H + ho0 - g.ph) * g.W) * g.C * 2;
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      const unsigned off = su[i] >= u_lo && su[i] < u_hi && sb[i] >= 0 ? (unsigned)(base + sb[i]) : 0x80000000u;
      rsl[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < DZ_PER; ++i) {
      const int e = i * NT + tid;
      if (e < DZ_N) *(uint4_t*)(dzs + (e >> 3) * RS + (e & 7) * 16) = rdz[i];
    }
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      const int e = i * NT + tid;
      if (e < Q::SL_N) *(uint4_t*)(sls + (e / SLC) * RSL + (e % SLC) * 16) = rsl[i];
    }
  };
  floatx4 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // column block cb = (ih, iw, 16-channel chunk cc) of this wave's three
  int cofs[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int cb = 3 * wave + j, ih = cb / (3 * CPT), iw = (cb % (3 * CPT)) / CPT, cc = cb % CPT;
    cofs[j] = (ih * Ls + iw) * RSL + cc * 32;
  }
  if (c_beg < c_end) {
    load(c_beg);
    store();
  }
  __syncthreads();
  for (int c = c_beg; c < c_end; ++c) {
    const bool more = c + 1 < c_end;
    const int kmax = (R * g.Wo + 31) / 32;   // 32-slot steps that can hold valid slots
    if (more) load(c + 1);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (kk < kmax) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const char* a = dzs + dz_off + 32 * kk * RS + i * 32;
          af[i] = wr::frag_at(a, a + 4 * RS);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const bf16x8 bf = wr::frag_at(sls + sl_off[kk][0] + cofs[j], sls + sl_off[kk][1] + cofs[j]);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (more) store();
    __syncthreads();
  }
  float* o = out + (long)split * Cout * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int cb = 3 * wave + j, ih = cb / (3 * CPT), iw = (cb % (3 * CPT)) / CPT, cc = cb % CPT;
      const long col = ((long)(it * g.kh + ih) * g.kw + iw) * g.C + ct * CS + cc * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cot * 64 + 16 * i + 4 * (lane >> 4) + r;
        o[(long)co * g.K + col] = acc[i][j][r];
      }
    }
}

// ---- forward (and stride-1 input gradient) of the k x k x 3 convolutions from input row slabs -------------------
// z[m, co] = Σ_(it, ih) Σ_iw Σ_c x[in(m, it, ih) + iw, c] · W[co, (it, ih, iw), c].  The generic kernel gathers one
// tap's 128 input rows per K-step; here a 256-row tile of M stages, per (it, ih, 64-channel slice), the input row
// segments of the output rows it touches ONCE (Ls = (Wo−1)·sw + 3 positions each) plus the three kw taps' weights,
// and the kw taps become row shifts of the slab: a third of the input gather per FLOP.  4 waves, each 64 rows x 64
// Cout of the tile (4 x 4 blocks of mfma_f32_16x16x32_bf16); LDS single-buffered with a register prefetch of the
// next step (2 workgroups per CU); 128-row BatchNorm tile statistics as conv3d_fwd_igemm's.
namespace fr {
constexpr int TN = 64, NT = 256, RS = 144;
// TM = 256 (4 waves x 64 rows, all 64 Cout each) or 128 (2 x 2 waves of 64 rows x 32 Cout: twice the workgroups for
// the small-M layers); SQ = slab rows for the output rows a tile can touch (1 + ⌈(TM−1)/Wo⌉ rows of Ls positions)
template <int TM> struct Cfg {
  static constexpr int WR = TM / 64, WC = 4 / WR, JB = 4 / WC, SQ = TM == 256 ? 352 : 184;
  static constexpr int SLAB = SQ * RS, WB = 3 * TN * RS;
  static constexpr int SL_PER = (SQ * 8 + NT - 1) / NT, W_PER = 3 * TN * 8 / NT, ELD = TN + 4;
  static constexpr int LDS = SLAB + WB + 2 * 64 * 4;   // + per-output-row table
  static_assert(TM * ELD * 4 + 2048 <= SLAB + WB, "epilogue staging + statistics scratch must fit the operand LDS");
};
}  // namespace fr

// raw (split-K over the (it, ih, 64-channel) K-steps, blockIdx.y = split of gridDim.y): this split's fp32 partial
// tile goes to raw[split][M][Cout] (no residual, rounding or statistics: conv_split_reduce finishes it).
template <int TM>
__global__ __launch_bounds__(256, 2) void conv3d_fwd_rows(Geom g, int M, int Cout, int Ls, const bf16* __restrict__ x,
                                                          const bf16* __restrict__ Wt, const bf16* __restrict__ res,
                                                          bf16* __restrict__ z, float* __restrict__ tstats,
                                                          float* __restrict__ raw = nullptr) {
  using namespace fr;
  typedef Cfg<TM> CF;
  constexpr int SQ = CF::SQ, SLAB = CF::SLAB, WB = CF::WB, SL_PER = CF::SL_PER, W_PER = CF::W_PER, ELD = CF::ELD;
  constexpr int JB = CF::JB;
  __shared__ __attribute__((aligned(16))) char smem[CF::LDS];
  char* const slab = smem;
  char* const wl = smem + SLAB;
  int* const tab = (int*)(smem + SLAB + WB);       // per output row r: [0][r] input-row base (position index),
                                                   // [1][r] t0 | h0 << 16 (biased by 0x8000)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave / CF::WC, wc = wave % CF::WC;
  const int tiles_n = Cout / TN, ntile = ((M + TM - 1) / TM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  const int bm = (bid / tiles_n) * TM, bn = (bid % tiles_n) * TN;
  const int rho_first = bm / g.Wo, rho_last = (min(M, bm + TM) - 1) / g.Wo, nr = rho_last - rho_first + 1;
  const int nq = nr * Ls;
  if (tid < nr) {
    const int rho = rho_first + tid;
    const int ho = rho % g.Ho, tn = rho / g.Ho, to = tn % g.To, n = tn / g.To;
    const int t0 = to * g.st - g.pt, h0 = ho * g.sh - g.ph;
    tab[tid] = ((n * g.T + t0) * g.H + h0) * g.W - g.pw;   // position of (t0, h0, w = −pw); t0/h0 may be negative
    tab[64 + tid] = (int)((unsigned)(t0 + 0x8000) | ((unsigned)(h0 + 0x8000) << 16));
  }
  // this thread's slab slots: (output row r, position) — fixed for the whole K loop
  int spos[SL_PER];
#pragma unroll
  for (int i = 0; i < SL_PER; ++i) {
    const int q = (i * NT + tid) >> 3;
    spos[i] = -1;
    if (q < nq) {
      const int r = q / Ls;
      spos[i] = (r << 8) | (q - r * Ls);
    }
  }
  // A fragment rows of this lane (slots 64·wave + 16i + lane&15 → slab row of tap iw = 0)
  int a_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = bm + 64 * wr + 16 * i + (lane & 15);
    const int row = m < M ? (m / g.Wo - rho_first) * Ls + (m % g.Wo) * g.sw : 0;
    a_off[i] = row * RS + (lane >> 4) * 16;
  }
  const int b_off = (lane & 15) * RS + (lane >> 4) * 16;
  const int ncc = g.C / 64, nks_all = g.kt * g.kh * ncc;
  const int split = blockIdx.y, nsp = gridDim.y;
  const int ks0 = (int)((long)nks_all * split / nsp), nks = (int)((long)nks_all * (split + 1) / nsp);
  uint4_t rsl[SL_PER], rw[W_PER];
  // operands through buffer resources with 32-bit byte offsets (the plan keeps x within 1 GiB); padding slots load
  // from offset 2^31, past the resource, which reads zeros (as conv3d_fwd_rows3)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);
  int wb[W_PER];   // this thread's weight pieces: byte offset of row bn + co, tap iw, channel chunk
#pragma unroll
  for (int i = 0; i < W_PER; ++i) {
    const int e = i * NT + tid, iw = e >> 9, co = (e >> 3) & 63, ch = e & 7;
    wb[i] = ((bn + co) * g.Kp + iw * g.C + ch * 8) * 2;
  }
  __syncthreads();   // the row table
  auto load = [&](int ks) {
    const int cc = ks % ncc, tap = ks / ncc, ih = tap % g.kh, it = tap / g.kh;
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      unsigned off = 0x80000000u;
      if (spos[i] >= 0) {
        const int r = spos[i] >> 8, pos = spos[i] & 255;
        const unsigned th = (unsigned)tab[64 + r];
        const int ti = (int)(th & 0xffffu) - 0x8000 + it, hi = (int)(th >> 16) - 0x8000 + ih, wi = pos - g.pw;
        if (ti >= 0 && ti < g.T && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
          off = (unsigned)(((tab[r] + (it * g.H + ih) * g.W + pos) * g.C + cc * 64 + ((i * NT + tid) & 7) * 8) * 2);
      }
      rsl[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
    const int so = (((it * g.kh + ih) * g.kw) * g.C + cc * 64) * 2;    // wave-uniform: the scalar offset
#pragma unroll
    for (int i = 0; i < W_PER; ++i)
      rw[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(wrs, wb[i], so, 0));
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      const int e = i * NT + tid, q = e >> 3, ch = e & 7;
      if (q < SQ) *(uint4_t*)(slab + q * RS + ch * 16) = rsl[i];
    }
#pragma unroll
    for (int i = 0; i < W_PER; ++i) {
      const int e = i * NT + tid;
      *(uint4_t*)(wl + (e >> 3) * RS + (e & 7) * 16) = rw[i];
    }
  };
  floatx4 acc[4][JB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  load(ks0);
  store();
  __syncthreads();
  for (int ks = ks0; ks < nks; ++ks) {
    const bool more = ks + 1 < nks;
    if (more) load(ks + 1);
    if (CMHAR_ROWS_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int iw = 0; iw < 3; ++iw)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4], bfr[JB];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(slab + a_off[i] + iw * RS + kk * 64);
#pragma unroll
        for (int j = 0; j < JB; ++j)
          bfr[j] = *(const bf16x8*)(wl + (iw * TN + 16 * JB * wc + 16 * j) * RS + b_off + kk * 64);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    if (CMHAR_ROWS_PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (more) store();
    __syncthreads();
  }
  // epilogue: fp32 tile through LDS, 8-column bf16 vectors (+ residual), then the 128-row BatchNorm tile statistics;
  // the residual rows are loaded before the staging (their latency paid once, not per row)
  uint4_t rq[TM / 32];
#pragma unroll
  for (int k = 0; k < TM / 32; ++k) {
    const int m = bm + (tid >> 3) + 32 * k;
    rq[k] = res && !raw && m < M ? *(const uint4_t*)(res + (long)m * Cout + bn + (tid & 7) * 8)
                                  : uint4_t{0u, 0u, 0u, 0u};
  }
  float* T = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(64 * wr + 16 * i + 4 * (lane >> 4) + r) * ELD + 16 * JB * wc + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int cg = (tid & 7) * 8;
#pragma unroll
  for (int k = 0; k < TM / 32; ++k) {
    const int rr = (tid >> 3) + 32 * k;
    const int m = bm + rr;
    if (m >= M) break;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = T[rr * ELD + cg + j];
    if (raw) {
      float* dst = raw + ((long)split * M + m) * Cout + bn + cg;
      *(floatx4*)dst = floatx4{v[0], v[1], v[2], v[3]};
      *(floatx4*)(dst + 4) = floatx4{v[4], v[5], v[6], v[7]};
      continue;
    }
    if (res) {
      const bf16x8 q = __builtin_bit_cast(bf16x8, rq[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)q[j];
    }
    zstore8(z + (long)m * Cout + bn + cg, v);
  }
  if (tstats && !raw) {
    // one statistics column per (128-row half, Cout column)
    const int ntm = (M + 127) / 128;
    tile_col_stats<NT>(
        (TM / 128) * TN, (float*)(smem + TM * ELD * 4), tid,
        [&](int w, int r) { return T[((w / TN) * 128 + r) * ELD + w % TN]; },
        [&](int w) { return min(128, M - (bm + (w / TN) * 128)); },
        [&](int w, float mu, float m2) {
          const int half = w / TN, c = w % TN, tm = bm / 128 + half;
          tstats[(long)tm * Cout + bn + c] = mu;
          tstats[((long)ntm + tm) * Cout + bn + c] = m2;
          if (c == 0 && bn == 0) tile_counts(tstats, ntm, Cout)[tm] = (float)min(128, M - (bm + half * 128));
        });
  }
}

// Split-K forward: z = Σ_split raw[split] (+ res), in split order, rounded once (conv3d_fwd_rows' epilogue
// arithmetic on the summed tile); 8 columns per thread.
__global__ __launch_bounds__(256) void conv_split_reduce(int M, int Cout, int nsplit, const float* __restrict__ raw,
                                                         const bf16* __restrict__ res, bf16* __restrict__ z) {
  const long n8 = (long)M * Cout / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long off = i * 8;
    float v[8];
    Vec8<float>::load(raw + off, v);
    for (int sp = 1; sp < nsplit; ++sp) {
      float w[8];
      Vec8<float>::load(raw + (long)sp * M * Cout + off, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += w[j];
    }
    if (res) {
      float r[8];
      Vec8<bf16>::load(res + off, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    zstore8(z + off, v);
  }
}

// Stride-1 H/W forward with all nine (ih, iw) taps per staged slab: a tile is R consecutive output rows of one
// frame (R·Wo <= 256, R balanced over the frame's rows) times one 64-wide Cout slice (the Cout slices of a frame
// tile are consecutive workgroup ids, so they share the input rows in one XCD's L2); per (it, 64-channel slice) it
// stages the R + 2 input row segments its rows read under any ih once, then the three kh taps' weights one after
// another (slab kept), so each staged input byte feeds 3·3 taps instead of 3 (the 256-row kernel restages per ih).
// Same 4-wave 64-slot x 64-Cout layout and register prefetch as conv3d_fwd_rows<256>; BatchNorm statistics per
// frame tile (its row count written by the first Cout slice).
// LDS images (SW): unpadded 128-B rows with the 16-B chunk c of row r stored at chunk (c ^ r) & 7.  The A fragment
// read (ds_read_b128: lanes 16 consecutive slab rows x 4 chunks, lane groups {0-3,12-15,20-27}, ... of
// MI355X_MICROARCH.md §LDS, bank (a/4) % 64) is then conflict-free when its 16 rows are consecutive and 2-way where
// they straddle an output row (the slab skips Ls - Wo = 2 rows there); the weight reads are conflict-free.  The
// 144-B padded rows (SW = false, CMHAR_ROWS3_SWZ=0) are 2-way on every A and B read and 2.5-3-way at row seams
// (2.4x the LDS read cycles; PMC: 55 bank-conflict cycles per 131 LDS-array cycles, gpurun_out/s2c_pmc_conv.txt).
namespace fr3 {
constexpr int SQ = 352, TN = 64, NT = 256, RS = 144, ELD = TN + 4;
constexpr int SL_PER = (SQ * 8 + NT - 1) / NT, W_PER = 3 * TN * 8 / NT;
template <bool SW> struct L {
  static constexpr int RB = SW ? 128 : RS;                       // bytes per LDS row
  static constexpr int SLAB = SQ * RB, WB = 3 * TN * RB, EPI = 256 * ELD * 4 + 2048;
  static constexpr int BYTES = SLAB + WB > EPI ? SLAB + WB : EPI;  // epilogue staging + statistics scratch overlay
  // byte offset of 16-B chunk c of row r
  static __device__ __forceinline__ int at(int r, int c) { return SW ? (r << 7) | (((r ^ c) & 7) << 4) : r * RS + c * 16; }
};
}  // namespace fr3

template <bool SW>
__global__ __launch_bounds__(256, 2) void conv3d_fwd_rows3(Geom g, int Cout, int R, int Ls, int cpf,
                                                           const bf16* __restrict__ x, const bf16* __restrict__ Wt,
                                                           const bf16* __restrict__ res, bf16* __restrict__ z,
                                                           float* __restrict__ tstats) {
  using namespace fr3;
  typedef fr3::L<SW> LY;
  __shared__ __attribute__((aligned(16))) char smem[LY::BYTES];
  char* const slab = smem;
  char* const wl = smem + LY::SLAB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncot = Cout / TN, ntile = gridDim.x / ncot;          // frame tiles
  const int tl = xcd_remap(blockIdx.x, gridDim.x);
  const int t = tl / ncot, bn = (tl - t * ncot) * TN;
  const int f = t / cpf, ho0 = (t - f * cpf) * R, nr = min(R, g.Ho - ho0);
  const int to = f % g.To, n = f / g.To;
  const int used = nr * g.Wo;
  const long m0 = ((long)f * g.Ho + ho0) * g.Wo;
  const int nq = (nr + 2) * Ls;
  // Operands through buffer resources with 32-bit byte offsets (the plan keeps x within 1 GiB): an offset past the
  // resource's range reads zeros, so the zero padding needs no select on the loaded value (a select right after a
  // prefetched load makes the compiler wait for it there) and no 64-bit address arithmetic per load.
  const unsigned xbytes = (unsigned)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);
  // block-invariant slab slots: byte offset of the slot's 16 B in frame ti = 0 of clip n (input row ho0 − ph + u,
  // u = 0..nr+1, and position), or 2^31 in the H / W padding or past the slab.  A load adds the group's frame offset
  // (< 2^30, or 2^30 for a frame in the T padding): every sum with a 2^30 / 2^31 term lies in [2^30, 2^32) — past the
  // resource's <= 2^30 bytes, so it reads zeros — and no select or branch is needed per load.
  unsigned pb[SL_PER];
#pragma unroll
  for (int i = 0; i < SL_PER; ++i) {
    const int q = (i * NT + tid) >> 3;
    const int u = q / Ls, wi = q - u * Ls - g.pw, hi = ho0 - g.ph + u;
    pb[i] = q < nq && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W
                ? (unsigned)(((((n * g.T) * g.H + hi) * g.W + wi) * g.C + ((i * NT + tid) & 7) * 8) * 2) : 0x80000000u;
  }
  // weight pieces of this thread: byte offset of row bn + co, tap iw, channel chunk (+ the stage's (it, ih, cc) part)
  int wb[W_PER];
#pragma unroll
  for (int i = 0; i < W_PER; ++i) {
    const int e = i * NT + tid, iw = e >> 9, co = (e >> 3) & 63, ch = e & 7;
    wb[i] = ((bn + co) * g.Kp + iw * g.C + ch * 8) * 2;
  }
  // A fragment rows of this lane (slots 64·wave + 16i + lane&15 → slab row of tap ih = iw = 0); its 16-B chunk
  // within a 64-B K half is lane >> 4
  const int cl = lane >> 4;
  int a_row[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 64 * wave + 16 * i + (lane & 15);
    a_row[i] = k < used ? (k / g.Wo) * Ls + (k % g.Wo) : 0;
  }
  const int b_off = LY::at(lane & 15, cl);        // weight row 16j + lane&15 of tap iw: + (iw·TN + 16j) rows
  const int ncc = g.C / 64, nst = g.kt * ncc * 3;
  uint4_t rsl[SL_PER], rw[W_PER];
  // stage s = (it, cc, ih), ih fastest; the slab changes with the group (it, cc), i.e. at ih = 0
  auto load_slab = [&](int grp) {
    const int cc = grp % ncc, it = grp / ncc;
    const int ti = to * g.st - g.pt + it;
    const bool tok = ti >= 0 && ti < g.T;
    const unsigned so = tok ? (unsigned)((ti * g.H * g.W * g.C + cc * 64) * 2) : 0x40000000u;
#pragma unroll
    for (int i = 0; i < SL_PER; ++i)
      rsl[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, pb[i] + so, 0, 0));
  };
  auto load_w = [&](int st) {
    const int ih = st % 3, cc = (st / 3) % ncc, it = st / (3 * ncc);
    const int so = (((it * g.kh + ih) * g.kw) * g.C + cc * 64) * 2;    // wave-uniform: the scalar offset
#pragma unroll
    for (int i = 0; i < W_PER; ++i)
      rw[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(wrs, wb[i], so, 0));
  };
  auto store_slab = [&]() {
#pragma unroll
    for (int i = 0; i < SL_PER; ++i) {
      const int e = i * NT + tid;
      if ((e >> 3) < SQ) *(uint4_t*)(slab + LY::at(e >> 3, e & 7)) = rsl[i];
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int i = 0; i < W_PER; ++i) {
      const int e = i * NT + tid;
      *(uint4_t*)(wl + LY::at(e >> 3, e & 7)) = rw[i];
    }
  };
  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int ih) {
    const int rsh = ih * Ls;                         // input row r + ih
#pragma unroll
    for (int iw = 0; iw < 3; ++iw)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4], bfr[4];
        // K half kk = chunks 4kk..4kk+3: chunk bit 2, i.e. byte-offset bit 6 of the swizzled address (rows are
        // 128 B, the XOR key only touches bits 4-6), or + 64 B on the padded rows
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *(const bf16x8*)(slab + (SW ? LY::at(a_row[i] + rsh + iw, cl) ^ (kk << 6)
                                               : LY::at(a_row[i] + rsh + iw, cl) + kk * 64));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = *(const bf16x8*)(wl + (iw * TN + 16 * j) * LY::RB + (SW ? b_off ^ (kk << 6) : b_off + kk * 64));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
  };
  load_slab(0);
  load_w(0);
  store_slab();
  store_w();
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    // the next stage's operands in registers during this stage's MFMAs (the slab only when the group changes);
    // loading the next group's slab at the group's first stage instead (three phases of prefetch) spilled
    // (256 VGPRs + 140 B scratch) and ran layer 1 at 738 vs 491 us
    const bool more = st + 1 < nst;
    if (more) {
      if ((st + 1) % 3 == 0) load_slab((st + 1) / 3);
      load_w(st + 1);
    }
    if (CMHAR_ROWS3_PRIO) __builtin_amdgcn_s_setprio(1);
    compute(st % 3);
    if (CMHAR_ROWS3_PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (more) {
      if ((st + 1) % 3 == 0) store_slab();
      store_w();
    }
    __syncthreads();
  }
  float* T = (float*)smem;
  const int cg = (tid & 7) * 8;
  // the residual (dgrad's dx_acc) rows of this thread, loaded before the accumulator staging: each load's latency
  // is then paid once, not once per row in the store loop (as the GEMM epilogues' streamed operands)
  uint4_t rq[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int rr = (tid >> 3) + 32 * k;
    rq[k] = res && rr < used ? *(const uint4_t*)(res + (m0 + rr) * Cout + bn + cg) : uint4_t{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(64 * wave + 16 * i + 4 * (lane >> 4) + r) * ELD + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int rr = (tid >> 3) + 32 * k;
    if (rr >= used) break;
    const long m = m0 + rr;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = T[rr * ELD + cg + j];
    if (res) {
      const bf16x8 q = __builtin_bit_cast(bf16x8, rq[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)q[j];
    }
    zstore8(z + m * Cout + bn + cg, v);
  }
  if (tstats)
    tile_col_stats<NT>(TN, (float*)(smem + 256 * ELD * 4), tid, [&](int c, int r) { return T[r * ELD + c]; },
                       [&](int) { return used; }, [&](int c, float mu, float m2) {
                         tstats[(long)t * Cout + bn + c] = mu;
                         tstats[((long)ntile + t) * Cout + bn + c] = m2;
                         if (c == 0 && bn == 0) tile_counts(tstats, ntile, Cout)[t] = (float)used;
                       });
}

// ---- implicit stem: few input channels (C <= 4), kw <= 8 taps at w-stride 2 (R3D-18's 3->64, 3x7x7, (1,2,2)) ----
// The generic path materialises a 448-wide bf16 column matrix (1.44 GB at B = 32) and multiplies it.  Here each
// (it, ih) tap row is ONE 32-wide K-step: an input row is staged in LDS as [position][4 channels] (8 B per position,
// channel 3 and the row padding zero), so the kw·4 window of output column wo starts at byte 16·wo — a 16-B
// aligned MFMA fragment read straight from the row (windows of neighbouring outputs overlap in LDS, no copy) — and
// the weights are packed [co][(it, ih)][iw·4 + c] with zeros at c >= C and iw >= kw (so the fragment's k beyond the
// window multiplies zero).  Tiles are up to R = ⌊256 / Wo⌋ output rows of one frame; per it the tile stages the
// (R−1)·sh + kh input rows its (row, ih) pairs read.  Forward and weight gradient; BatchNorm tile statistics as the
// row-slab kernels.
namespace stm {
constexpr int RB = 16 * 64 + 16;      // LDS bytes per staged input row (<= 127 positions x 8 B, + pad)
constexpr int UMAX = 13, KHMAX = 8, WCO = 80;   // staged rows per tile, kh taps, weight row stride (64 B + pad)
constexpr int ROWS_B = UMAX * RB, W_B = KHMAX * 64 * WCO, ELD = 68;
constexpr int FWD_LDS = (ROWS_B + W_B) > 256 * ELD * 4 + 2048 ? (ROWS_B + W_B) : 256 * ELD * 4 + 2048;
__device__ __forceinline__ bool ok(const Geom& g) { return g.C <= 4 && g.kw <= 8 && g.sw == 2 && g.kh <= KHMAX; }
}  // namespace stm

__global__ __launch_bounds__(256, 2) void conv3d_stem_fwd(Geom g, int R, int cpf, const bf16* __restrict__ x,
                                                          const bf16* __restrict__ W4, bf16* __restrict__ z,
                                                          float* __restrict__ tstats) {
  using namespace stm;
  __shared__ __attribute__((aligned(16))) char smem[FWD_LDS];
  char* const rows = smem;
  char* const wl = smem + ROWS_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntile = gridDim.x;
  const int t = xcd_remap(blockIdx.x, ntile);
  const int f = t / cpf, ho0 = (t - f * cpf) * R, nr = min(R, g.Ho - ho0);
  const int to = f % g.To, n = f / g.To;
  const int used = nr * g.Wo, U = (nr - 1) * g.sh + g.kh, Lrow = (g.Wo - 1) * g.sw + 8;
  const long m0 = ((long)f * g.Ho + ho0) * g.Wo;
  const int G = g.kh * 32;   // weight elements per (co, it)
  int a_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 64 * wave + 16 * i + (lane & 15);
    a_off[i] = (k < used ? (k / g.Wo) * g.sh * RB + (k % g.Wo) * 16 : 0) + (lane >> 4) * 16;
  }
  const int b_off = (lane & 15) * WCO + (lane >> 4) * 16;
  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Tap plane it + 1 (its input rows and weights) is loaded into registers while plane it is multiplied, through
  // buffer resources: a padding position / channel reads from offset 2^31, past the resource, which returns zero —
  // no select on the loaded values (which would make the compiler wait for the loads right there) and 32-bit offsets.
  constexpr int RPT = (UMAX * ((RB - 16) / 8) + 255) / 256, WPT = KHMAX * 64 * 4 / 256;
  const int nel = U * Lrow;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)W4, (short)0, 0x7fffffff, 0x00020000);
  int lo[RPT], go[RPT];   // staged position e = k·256 + tid: LDS byte offset (-1: none); input byte offset in
                          // frame ti = 0 of clip n (-1: H / W padding)
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int e = k * 256 + tid, u = e / Lrow, pp = e - u * Lrow, hi = ho0 * g.sh - g.ph + u, wi = pp - g.pw;
    lo[k] = e < nel ? u * RB + pp * 8 : -1;
    go[k] = e < nel && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W ? (((n * g.T) * g.H + hi) * g.W + wi) * g.C * 2 : -1;
  }
  unsigned short rx[RPT][4];
  uint4_t rwt[WPT];
  auto load_plane = [&](int it) {
    const int ti = to * g.st - g.pt + it;
    const bool tok = ti >= 0 && ti < g.T;
    const int fo = ti * g.H * g.W * g.C * 2;
    // out of range: bit 31 set on the offset (branch-free; a valid offset is < 2^31, an invalid one lands in
    // [2^31, 2^32), past the resource)
#pragma unroll
    for (int k = 0; k < RPT; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        rx[k][c] = __builtin_amdgcn_raw_buffer_load_b16(
            xr, (unsigned)(go[k] + fo + 2 * c) | ((unsigned)!(tok && go[k] >= 0 && c < g.C) << 31), 0, 0);
#pragma unroll
    for (int k = 0; k < WPT; ++k) {                        // [ih][co][4 x 16 B]
      const int e = k * 256 + tid, ih = e >> 8, co = (e >> 2) & 63, q = e & 3;
      rwt[k] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(
          wrs, (unsigned)(((co * g.kt + it) * G + ih * 32 + q * 8) * 2) | ((unsigned)(ih >= g.kh) << 31), 0, 0));
    }
  };
  auto store_plane = [&]() {
#pragma unroll
    for (int k = 0; k < RPT; ++k)
      if (lo[k] >= 0)
        *(short4_t*)(rows + lo[k]) = short4_t{(short)rx[k][0], (short)rx[k][1], (short)rx[k][2], (short)rx[k][3]};
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
      const int e = k * 256 + tid, ih = e >> 8, co = (e >> 2) & 63, q = e & 3;
      if (ih < g.kh) *(uint4_t*)(wl + (ih * 64 + co) * WCO + q * 16) = rwt[k];
    }
  };
  load_plane(0);
  for (int it = 0; it < g.kt; ++it) {
    if (it) __syncthreads();      // the previous plane's reads are done
    store_plane();
    __syncthreads();
    if (it + 1 < g.kt) load_plane(it + 1);
    for (int ih = 0; ih < g.kh; ++ih) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(rows + a_off[i] + ih * RB);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *(const bf16x8*)(wl + (ih * 64 + 16 * j) * WCO + b_off);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();
  float* T = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(64 * wave + 16 * i + 4 * (lane >> 4) + r) * ELD + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int cg = (tid & 7) * 8;
  for (int rr = tid >> 3; rr < used; rr += 32) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = T[rr * ELD + cg + j];
    zstore8(z + (m0 + rr) * 64 + cg, v);
  }
  if (tstats)
    tile_col_stats<256>(64, (float*)(smem + 256 * ELD * 4), tid, [&](int c, int r) { return T[r * ELD + c]; },
                        [&](int) { return used; }, [&](int c, float mu, float m2) {
                          tstats[(long)t * 64 + c] = mu;
                          tstats[((long)ntile + t) * 64 + c] = m2;
                          if (c == 0) tile_counts(tstats, ntile, 64)[t] = (float)used;
                        });
}

// Weight gradient dW4[co][it][ih][iw·4 + c] = Σ_slots dz[slot][co] · window(slot, it, ih)[iw·4 + c]: workgroup =
// (it, split of the tiles), wave = ih (2 column blocks of 16 x 4 Cout blocks); per tile it stages dz [256 slots][64]
// and the tile's input rows for plane it, and reads the window columns transposed (rows = slots, 16 B apart).
constexpr int STW_DZ = 256 * 144;
__global__ __launch_bounds__(512, 1) void conv3d_stem_wgrad(Geom g, int R, int cpf, int ntile, int tiles_per_split,
                                                            const bf16* __restrict__ x, const bf16* __restrict__ dz,
                                                            float* __restrict__ out) {
  using namespace stm;
  __shared__ __attribute__((aligned(16))) char smem[STW_DZ + ROWS_B];
  char* const dzs = smem;
  char* const rows = smem + STW_DZ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nt = blockDim.x;
  const int it = blockIdx.x, split = blockIdx.y;
  const int t_beg = split * tiles_per_split, t_end = min(ntile, t_beg + tiles_per_split);
  const int Lrow = (g.Wo - 1) * g.sw + 8, G = g.kh * 32;
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p = lane & 3;
  const int lane_col = (p >> 1) * 16 + (p & 1) * 8;
  const bool active = wave < g.kh;
  floatx4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // The tile's loads (dz rows, input rows of plane it) are all issued before its LDS stores, through buffer resources
  // with out-of-range offsets (bit 31) for the padding, which read zero: the select after each dz load and the branch
  // around each input load made every load wait for the one before.  (A register pipeline one tile ahead measured
  // 355 -> 459 us per launch in the step trace; this keeps the synchronous staging.)
  constexpr int NTW = 64 * KHMAX, DPT = 256 * 8 / NTW, RPT = (UMAX * ((RB - 16) / 8) + NTW - 1) / NTW;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)min((long)g.N * g.T * g.H * g.W * g.C * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t dzr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dz, (short)0, (int)min((long)g.N * g.To * g.Ho * g.Wo * 64 * 2, 0x7fffffffL), 0x00020000);
  for (int t = t_beg; t < t_end; ++t) {
    const int f = t / cpf, ho0 = (t - f * cpf) * R, nr = min(R, g.Ho - ho0);
    const int to = f % g.To, n = f / g.To;
    const int used = nr * g.Wo, U = (nr - 1) * g.sh + g.kh, nel = U * Lrow;
    const int m0 = (f * g.Ho + ho0) * g.Wo;
    uint4_t rdz[DPT];
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = k * NTW + tid, j = e >> 3, ch = e & 7;
      rdz[k] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(
          dzr, (unsigned)(((m0 + j) * 64 + ch * 8) * 2) | ((unsigned)(j >= used) << 31), 0, 0));
    }
    const int ti = to * g.st - g.pt + it;
    const bool tok = ti >= 0 && ti < g.T;
    unsigned short rx[RPT][4];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = k * NTW + tid, u = e / Lrow, pp = e - u * Lrow, hi = ho0 * g.sh - g.ph + u, wi = pp - g.pw;
      const bool pok = tok && e < nel && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      const int go = (((n * g.T + ti) * g.H + hi) * g.W + wi) * g.C * 2;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        rx[k][c] = __builtin_amdgcn_raw_buffer_load_b16(xr, (unsigned)(go + 2 * c) | ((unsigned)!(pok && c < g.C) << 31),
                                                        0, 0);
    }
    if (t > t_beg) __syncthreads();
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = k * NTW + tid, j = e >> 3, ch = e & 7;
      *(uint4_t*)(dzs + j * 144 + ch * 16) = rdz[k];
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = k * NTW + tid, u = e / Lrow, pp = e - u * Lrow;
      if (e < nel)
        *(short4_t*)(rows + u * RB + pp * 8) = short4_t{(short)rx[k][0], (short)rx[k][1], (short)rx[k][2], (short)rx[k][3]};
    }
    __syncthreads();
    if (active) {
      const int kmax = (used + 31) / 32;
      for (int kk = 0; kk < kmax; ++kk) {
        const int k_lo = 32 * kk + 8 * gq + q4, k_hi = k_lo + 4;
        const int r_lo = k_lo < used ? (k_lo / g.Wo) * g.sh * RB + (k_lo % g.Wo) * 16 : 0;
        const int r_hi = k_hi < used ? (k_hi / g.Wo) * g.sh * RB + (k_hi % g.Wo) * 16 : 0;
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const char* a = dzs + (32 * kk + 8 * gq + q4) * 144 + lane_col + i * 32;
          af[i] = wr::frag_at(a, a + 4 * 144);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const char* b = rows + wave * RB + lane_col + 32 * j;
          const bf16x8 bf = wr::frag_at(b + r_lo, b + r_hi);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  if (!active) return;
  float* o = out + (long)split * 64 * g.kt * G;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * i + 4 * (lane >> 4) + r;
        o[(long)co * g.kt * G + it * G + wave * 32 + 16 * j + (lane & 15)] = acc[i][j][r];
      }
}

// [Cout][C][kt][kh][kw] fp32 → [Cout][kt][kh][32] bf16 with element iw·4 + c (zero past kw / C)
__global__ void stem_pack_kernel(int Cout, int C, int kt, int kh, int kw, const float* __restrict__ w,
                                 bf16* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, G = kh * 32;
  if (i >= Cout * kt * G) return;
  const int co = i / (kt * G), r = i % (kt * G), it = r / G, ih = (r % G) / 32, e = r % 32, iw = e >> 2, c = e & 3;
  out[i] = (iw < kw && c < C) ? (bf16)w[((((long)co * C + c) * kt + it) * kh + ih) * kw + iw] : (bf16)0.f;
}

// dW = Σ_z ws[z] in a fixed order (deterministic), 4 floats per thread.  The slices are loaded four at a time before
// they are added in order (one load in flight per wave left the kernel latency-bound at 1.8 TB/s).
__global__ __launch_bounds__(256) void conv3d_wgrad_reduce(long n4, int splits, long slab, const float* __restrict__ ws,
                                                           float* __restrict__ dw) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    floatx4 s = *(const floatx4*)(ws + i * 4);
    int z = 1;
    for (; z + 3 < splits; z += 4) {
      floatx4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const floatx4*)(ws + (z + u) * slab + i * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; z < splits; ++z) s += *(const floatx4*)(ws + z * slab + i * 4);
    *(floatx4*)(dw + i * 4) = s;
  }
}

inline int grid_for(long work) {
  const long b = (work + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

inline bool bn_channels_ok(int C) { return C >= 8 && C % 8 == 0 && C <= 2048; }

// ≤ 1024 chunks of ≥ 16 K elements per tensor: four blocks per CU stream the big R3D-18 layers (M·C = 103 M at
// 16×56², where ≤ 512 chunks of ≥ 512 rows ran 1.5 TB/s), a few blocks the 7² layer-4 maps; few partials to combine
inline int bn_chunks(long M, int C) {
  const long c = (M * C + 16383) / 16384;
  return (int)(c < 1024 ? (c > 0 ? c : 1) : 1024);
}

Geom make_geom(const int* dims) {
  Geom g;
  g.N = dims[0]; g.T = dims[1]; g.H = dims[2]; g.W = dims[3]; g.C = dims[4];
  g.kt = dims[5]; g.kh = dims[6]; g.kw = dims[7];
  g.st = dims[8]; g.sh = dims[9]; g.sw = dims[10];
  g.pt = dims[11]; g.ph = dims[12]; g.pw = dims[13];
  g.To = (g.T + 2 * g.pt - g.kt) / g.st + 1;
  g.Ho = (g.H + 2 * g.ph - g.kh) / g.sh + 1;
  g.Wo = (g.W + 2 * g.pw - g.kw) / g.sw + 1;
  g.K = g.kt * g.kh * g.kw * g.C;
  g.Kp = dims[14];
  return g;
}

bool geom_ok(const Geom& g) {
  return g.N > 0 && g.T > 0 && g.H > 0 && g.W > 0 && g.C > 0 && g.kt > 0 && g.kh > 0 && g.kw > 0 && g.st > 0 &&
         g.sh > 0 && g.sw > 0 && g.pt >= 0 && g.ph >= 0 && g.pw >= 0 && g.To > 0 && g.Ho > 0 && g.Wo > 0 &&
         g.Kp >= g.K;
}

}  // namespace

extern "C" int cmhar_conv3d_im2col(int in_dtype, int out_dtype, const int* dims, const void* x, void* col,
                                   hipStream_t stream) {
  const Geom g = make_geom(dims);
  if (!geom_ok(g)) return -1;
  const long Ml = (long)g.N * g.To * g.Ho * g.Wo;
  if (Ml >= (1L << 31) || (long)g.N * g.T * g.H * g.W >= (1L << 31)) return -2;
  const int M = (int)Ml;
  const bool vec = g.C % 8 == 0 && g.Kp % 8 == 0;
  const int kv = vec ? g.Kp / 8 : g.Kp;
  int tpr = 1;
  while (tpr < kv && tpr < 256) tpr <<= 1;
  const int rows_grid = grid_for((long)M * tpr);
#define IM2COL(TI, TO)                                                                                          \
  do {                                                                                                          \
    if (vec) im2col3d_kernel<TI, TO, 8><<<rows_grid, 256, 0, stream>>>(g, M, tpr, (const TI*)x, (TO*)col);     \
    else if (g.Kp % 8 == 0)                                                                                   \
      im2col3d_vec_store_kernel<TI, TO><<<grid_for((long)M * (g.Kp / 8)), 256, 0, stream>>>(g, M, (const TI*)x, \
                                                                                             (TO*)col);        \
    else im2col3d_kernel<TI, TO, 1><<<rows_grid, 256, 0, stream>>>(g, M, tpr, (const TI*)x, (TO*)col);         \
  } while (0)
  if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_BF16) IM2COL(bf16, bf16);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_F32) IM2COL(float, float);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_BF16) IM2COL(float, bf16);
  else return -1;
#undef IM2COL
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_conv3d_col2im(int dtype, const int* dims, const void* dcol, void* dx, int accumulate,
                                   hipStream_t stream) {
  const Geom g = make_geom(dims);
  if (!geom_ok(g)) return -1;
  if ((long)g.N * g.T * g.H * g.W * g.C >= (1L << 32) || (long)g.N * g.To * g.Ho * g.Wo >= (1L << 31)) return -2;
  const bool vec = g.C % 8 == 0;
  const long work = (long)g.N * g.T * g.H * g.W * (vec ? g.C / 8 : g.C);
  const int grid = grid_for(work);
  const int mt = max(max(cdiv(g.kt, g.st), cdiv(g.kh, g.sh)), cdiv(g.kw, g.sw));
  const bool gather = dtype == CMHAR_BF16 && vec && mt <= 3 && (long)g.N * g.To * g.Ho * g.Wo * g.Kp * 2 < (1L << 31);
  if (gather) {
    if (mt == 1) col2im3d_gather<1><<<grid, 256, 0, stream>>>(g, (const bf16*)dcol, (bf16*)dx, accumulate);
    else if (mt == 2) col2im3d_gather<2><<<grid, 256, 0, stream>>>(g, (const bf16*)dcol, (bf16*)dx, accumulate);
    else col2im3d_gather<3><<<grid, 256, 0, stream>>>(g, (const bf16*)dcol, (bf16*)dx, accumulate);
  } else if (dtype == CMHAR_BF16) {
    if (vec) col2im3d_kernel<bf16, 8><<<grid, 256, 0, stream>>>(g, (const bf16*)dcol, (bf16*)dx, accumulate);
    else col2im3d_kernel<bf16, 1><<<grid, 256, 0, stream>>>(g, (const bf16*)dcol, (bf16*)dx, accumulate);
  } else if (dtype == CMHAR_F32) {
    if (vec) col2im3d_kernel<float, 8><<<grid, 256, 0, stream>>>(g, (const float*)dcol, (float*)dx, accumulate);
    else col2im3d_kernel<float, 1><<<grid, 256, 0, stream>>>(g, (const float*)dcol, (float*)dx, accumulate);
  } else {
    return -1;
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// A thread's 8 channels are fixed along the grid-stride loop when C/8 divides 256 (grid_for's blocks are 256 wide)
inline bool bn_hoist(int C) { return 256 % (C / 8) == 0; }

template <typename T>
void bn_apply_launch(long M, int C, const void* x, const void* res, const float* smean, const float* srstd,
                     const float* w, const float* b, int relu, void* y, hipStream_t stream) {
  const unsigned nvec = (unsigned)(M * C / 8);
  if (bn_hoist(C))
    bn_cl_apply<T, true><<<grid_for(nvec), 256, 0, stream>>>(nvec, C, (const T*)x, (const T*)res, smean, srstd, w,
                                                              b, relu, (T*)y);
  else
    bn_cl_apply<T, false><<<grid_for(nvec), 256, 0, stream>>>(nvec, C, (const T*)x, (const T*)res, smean, srstd, w,
                                                               b, relu, (T*)y);
}

// BatchNorm backward: column partials (Σg, Σg·x̂), their combination into db / dw, then dx (and dres).
// y == nullptr with relu != 0: no residual entered the unit, the activation mask is recomputed from x (BN_ZMASK).
template <typename T>
int bn_bwd_launch(long M, int C, const void* x, const void* y, const void* dy, const float* w, const float* b,
                  const float* smean, const float* srstd, void* dx, void* dres, float* dw, float* db, int training,
                  int relu, float* ws, hipStream_t stream) {
  const int nch = bn_chunks(M, C);
  const int rpc = (int)((M + nch - 1) / nch);
  const int act = relu && !y ? relu | BN_ZMASK : relu;
  if (act & BN_ZMASK)
    bn_cl_partial<T, 2, true><<<nch, 256, 0, stream>>>((int)M, C, rpc, (const T*)x, (const T*)y, (const T*)dy, smean,
                                                     srstd, w, b, act, ws);
  else
    bn_cl_partial<T, 2, false><<<nch, 256, 0, stream>>>((int)M, C, rpc, (const T*)x, (const T*)y, (const T*)dy,
                                                      smean, srstd, w, b, act, ws);
  bn_cl_final<<<(C + BN_FC - 1) / BN_FC, 256, 0, stream>>>(2, M, C, nch, ws, nullptr, nullptr, nullptr, nullptr,
                                                           nullptr, 0.f, 0.f, dw, db);
  const unsigned nvec = (unsigned)(M * C / 8);
  if (bn_hoist(C))
    bn_cl_bwd_apply<T, true><<<grid_for(nvec), 256, 0, stream>>>(nvec, (int)M, C, (const T*)x, (const T*)y,
                                                                  (const T*)dy, smean, srstd, w, b, dw, db, training,
                                                                  act, (T*)dx, (T*)dres);
  else
    bn_cl_bwd_apply<T, false><<<grid_for(nvec), 256, 0, stream>>>(nvec, (int)M, C, (const T*)x, (const T*)y,
                                                                   (const T*)dy, smean, srstd, w, b, dw, db, training,
                                                                   act, (T*)dx, (T*)dres);
  return 0;
}

extern "C" long cmhar_bn_cl_ws(long M, int C) { return 2L * bn_chunks(M, C) * C; }

extern "C" int cmhar_bn_cl_fwd(int dtype, long M, int C, const void* x, const void* res, void* y, const float* w,
                               const float* b, float* rmean, float* rvar, float* smean, float* srstd, int training,
                               float momentum, float eps, int relu, long long* num_batches_tracked, float* ws,
                               hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !ws) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 31)) return -2;   // unsigned grid-stride loops never wrap
  const int nch = bn_chunks(M, C);
  const int rpc = (int)((M + nch - 1) / nch);
  const int fgrid = (C + BN_FC - 1) / BN_FC;
  if (training) {
    for (int mode = 0; mode < 2; ++mode) {
#define BNP(T, MODE)                                                                                            \
  bn_cl_partial<T, MODE><<<nch, 256, 0, stream>>>((int)M, C, rpc, (const T*)x, nullptr, nullptr, smean, nullptr,  \
                                                  nullptr, nullptr, 0, ws)
      if (dtype == CMHAR_BF16) {
        if (mode == 0) BNP(bf16, 0);
        else BNP(bf16, 1);
      } else if (dtype == CMHAR_F32) {
        if (mode == 0) BNP(float, 0);
        else BNP(float, 1);
      } else return -1;
#undef BNP
      bn_cl_final<<<fgrid, 256, 0, stream>>>(mode, M, C, nch, ws, smean, srstd, rmean, rvar, num_batches_tracked,
                                             momentum, eps, nullptr, nullptr);
    }
  } else {
    if (!rmean || !rvar) return -2;
    bn_cl_eval_stats<<<(C + 255) / 256, 256, 0, stream>>>(C, rmean, rvar, eps, smean, srstd);
  }
  if (dtype == CMHAR_BF16) bn_apply_launch<bf16>(M, C, x, res, smean, srstd, w, b, relu, y, stream);
  else bn_apply_launch<float>(M, C, x, res, smean, srstd, w, b, relu, y, stream);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_bn_cl_fwd_tiles(long M, int C, int ntile, float* tile_stats, const void* x, const void* res,
                                     void* y, const float* w, const float* b, float* rmean, float* rvar,
                                     float* smean, float* srstd, float momentum, float eps, int relu,
                                     long long* num_batches_tracked, hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !tile_stats || ntile <= 0) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 31)) return -2;   // unsigned grid-stride loops never wrap
  const int ngroup = (ntile + BN_TG - 1) / BN_TG;
  float* groups = (float*)tile_stats + 2L * ntile * C;
  const float* cnt = (float*)tile_stats + 2L * (ntile + ngroup) * C;
  float* gcnt = (float*)cnt + ntile;
  bn_tile_group<<<cdiv((long)ngroup * C, 256), 256, 0, stream>>>(C, ntile, tile_stats, cnt, groups, gcnt);
  bn_tile_final<<<(C + BN_GC - 1) / BN_GC, 256, 0, stream>>>(M, C, ngroup, groups, gcnt, smean, srstd, rmean, rvar,
                                                   num_batches_tracked, momentum, eps);
  bn_apply_launch<bf16>(M, C, x, res, smean, srstd, w, b, relu, y, stream);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_bn_cl_bwd(int dtype, long M, int C, const void* x, const void* y, const void* dy,
                               const float* w, const float* smean, const float* srstd, void* dx, void* dres,
                               float* dw, float* db, int training, int relu, float* ws, hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !ws || !dw || !db || (relu && !y)) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 31)) return -2;   // unsigned grid-stride loops never wrap
  if (dtype == CMHAR_BF16)
    bn_bwd_launch<bf16>(M, C, x, y, dy, w, nullptr, smean, srstd, dx, dres, dw, db, training, relu, ws, stream);
  else if (dtype == CMHAR_F32)
    bn_bwd_launch<float>(M, C, x, y, dy, w, nullptr, smean, srstd, dx, dres, dw, db, training, relu, ws, stream);
  else return -1;
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_bn_cl_bwd_nores(int dtype, long M, int C, const void* x, const void* dy, const float* w,
                                     const float* b, const float* smean, const float* srstd, void* dx, float* dw,
                                     float* db, int training, int relu, float* ws, hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !ws || !dw || !db || relu < 0 || relu > 2 || (relu && !b)) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 31)) return -2;   // unsigned grid-stride loops never wrap
  if (dtype == CMHAR_BF16)
    bn_bwd_launch<bf16>(M, C, x, nullptr, dy, w, b, smean, srstd, dx, nullptr, dw, db, training, relu, ws, stream);
  else if (dtype == CMHAR_F32)
    bn_bwd_launch<float>(M, C, x, nullptr, dy, w, b, smean, srstd, dx, nullptr, dw, db, training, relu, ws, stream);
  else return -1;
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_avgpool_cl(int dtype, int N, long S, int C, const void* x, float* out, hipStream_t stream) {
  if (N <= 0 || S <= 0 || !bn_channels_ok(C)) return -1;
  const int CB = C < 256 ? C : 256;
  dim3 grid(cdiv(C, CB), N);
  if (dtype == CMHAR_BF16) avgpool_cl_fwd<bf16><<<grid, 256, 0, stream>>>(N, S, C, (const bf16*)x, out);
  else if (dtype == CMHAR_F32) avgpool_cl_fwd<float><<<grid, 256, 0, stream>>>(N, S, C, (const float*)x, out);
  else return -1;
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_avgpool_cl_bwd(int dtype, int N, long S, int C, const float* dout, void* dx,
                                    hipStream_t stream) {
  if (N <= 0 || S <= 0 || C <= 0) return -1;
  const long total = (long)N * S * C;
  if (dtype == CMHAR_BF16) avgpool_cl_bwd<bf16><<<grid_for(total), 256, 0, stream>>>(total, S, C, dout, (bf16*)dx);
  else if (dtype == CMHAR_F32)
    avgpool_cl_bwd<float><<<grid_for(total), 256, 0, stream>>>(total, S, C, dout, (float*)dx);
  else return -1;
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_video_to_ndhwc(int out_dtype, int B, int T, int C, int H, int W, const float* video, void* out,
                                    hipStream_t stream) {
  if (B <= 0 || T <= 0 || C <= 0 || H <= 0 || W <= 0) return -1;
  const long total = (long)B * T * C * H * W, HW = (long)H * W;
  if (out_dtype == CMHAR_BF16)
    video_ndhwc_kernel<bf16><<<grid_for(total), 256, 0, stream>>>(total, C, HW, video, (bf16*)out);
  else if (out_dtype == CMHAR_F32)
    video_ndhwc_kernel<float><<<grid_for(total), 256, 0, stream>>>(total, C, HW, video, (float*)out);
  else return -1;
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// ---- implicit-GEMM entry points (bf16, C % 64 == 0, Kp == kt·kh·kw·C) ----
static bool igemm_ok(const Geom& g, int Cout) {
  return geom_ok(g) && g.C % 64 == 0 && g.Kp == g.K && Cout > 0 && Cout % 8 == 0 &&
         (long)g.N * g.To * g.Ho * g.Wo < (1L << 31);
}

// Statistics tiles the forward plan writes (see cmhar_conv3d_fwd; all its kernels use 128-row tiles) and the floats
// the caller provides for them: tile and group partials plus their row counts.
// Nine-tap forward (conv3d_fwd_rows3) plan: Cout % 64 == 0, 3x3 taps at unit H/W stride, R + 2 input rows of a
// tile in the slab, R = ⌈Ho / cpf⌉ with cpf = ⌈Ho / ⌊256 / Wo⌋⌉ tiles per frame (balanced: R3D-18 layer 2 takes
// 4 x 7 rows, not 9 + 9 + 9 + 1), and at least 3/4 of the tile's 256 MFMA row slots used (layer 4's 7 x 7 frames
// would use 49: it keeps the split-K row-slab kernel).  ntile counts frame tiles; the grid is ntile x Cout / 64.
// CMHAR_FWD_ROWS3=0 turns it off, =1 keeps it to Cout = 64 (R3D-18 layer 1 only; A/B runs).
struct Fwd3Plan { int R, Ls, cpf, ntile; };
static bool fwd3_plan(const Geom& g, int Cout, Fwd3Plan& p) {
  static const int mode = [] {
    const char* v = getenv("CMHAR_FWD_ROWS3");
    return v && (v[0] == '0' || v[0] == '1') ? v[0] - '0' : 2;
  }();
  if (!mode || (mode == 1 && Cout != fr3::TN) || Cout % fr3::TN || g.kh != 3 || g.kw != 3 || g.sh != 1 ||
      g.sw != 1 || g.C % 64 || g.Wo > 256 || (long)g.N * g.T * g.H * g.W * g.C * 2 > (1L << 30) ||
      (long)Cout * g.Kp * 2 > 0x7fffffffL)   // 32-bit buffer offsets of x (<= 1 GiB) and of the weights
    return false;
  const int r0 = min(256 / g.Wo, g.Ho);
  p.cpf = (g.Ho + r0 - 1) / r0;
  p.R = (g.Ho + p.cpf - 1) / p.cpf;
  p.Ls = g.Wo - 1 + g.kw;
  if ((p.R + 2) * p.Ls > fr3::SQ || 4 * p.R * g.Wo < 3 * 256 || (p.cpf - 1) * p.R >= g.Ho) return false;
  p.ntile = g.N * g.To * p.cpf;
  return true;
}
static int fwd_stat_tiles(const Geom& g, int M, int Cout) {
  Fwd3Plan p;
  if (fwd3_plan(g, Cout, p)) return p.ntile;
  return (M + 127) / 128;
}
extern "C" int cmhar_conv3d_fwd_tiles(const int* dims, int Cout) {
  const Geom g = make_geom(dims);
  if (!igemm_ok(g, Cout)) return -1;
  return fwd_stat_tiles(g, g.N * g.To * g.Ho * g.Wo, Cout);
}
extern "C" long cmhar_conv3d_fwd_stats_floats(const int* dims, int Cout) {
  const int nt = cmhar_conv3d_fwd_tiles(dims, Cout);
  if (nt <= 0) return -1;
  const int ng = (nt + BN_TG - 1) / BN_TG;
  return 2L * (nt + ng) * Cout + nt + ng;
}

// Split-K plan for the forward convs whose 128-row tile grid leaves most of the chip idle (R3D-18 layer 4: 3136 rows
// × 512 outputs = 200 tiles for 512 workgroup slots): the (it, ih, channel-slice) K-steps split over nsplit workgroups
// per tile, fp32 partials in the caller's workspace, conv_split_reduce sums them in order (+ residual) and rounds
// once.  No BatchNorm tile statistics (the caller takes the statistics passes over z: small at these sizes).
// 0 = not this plan.  CMHAR_FWD_SPLIT=0 turns it off (A/B runs).
// The generic implicit GEMM (strided convs: R3D-18 layer 4's stride-2 3x3 conv, 3136 x 512 = 100 128x128 tiles, and
// its 1x1 downsample) splits the same way over its BK-wide K-steps: split y takes kps of them (ig_split_kps).
static int fwd_plan(const Geom& g, int Cout);
static bool fwd_split_on() {
  static const bool on = [] {
    const char* v = getenv("CMHAR_FWD_SPLIT");
    return !(v && v[0] == '0');
  }();
  return on;
}
static int ig_split_count(const Geom& g, int Cout, int& kps) {
  kps = 0;
  if (!fwd_split_on() || !igemm_ok(g, Cout)) return 0;
  const int plan = fwd_plan(g, Cout);
  if ((plan != 4 && plan != 5) || (long)g.N * g.T * g.H * g.W * g.C * 2 > 0x7fffffffL ||
      (long)Cout * g.Kp * 2 > 0x7fffffffL)   // the buffer-resource instantiation only
    return 0;
  const int M = g.N * g.To * g.Ho * g.Wo;
  const long tiles = (long)((M + 127) / 128) * (plan == 4 ? 1 : (Cout + 127) / 128);
  if (tiles >= 256) return 0;
  const int nk = g.K / ig::BK;
  const int s0 = (int)std::min<long>(4, (512 + tiles - 1) / tiles);
  if (s0 < 2 || nk < 2 * s0) return 0;
  kps = (nk + s0 - 1) / s0;
  return (nk + kps - 1) / kps;   // every split non-empty
}
static int fwd_split_count(const Geom& g, int Cout) {
  if (!fwd_split_on() || !igemm_ok(g, Cout)) return 0;
  int kps;
  if (const int s = ig_split_count(g, Cout, kps)) return s;
  Fwd3Plan p3;
  if (fwd3_plan(g, Cout, p3)) return 0;
  const int M = g.N * g.To * g.Ho * g.Wo;
  const int Ls = (g.Wo - 1) * g.sw + g.kw;
  if (g.kw != 3 || Cout % fr::TN || g.Wo > 255 || Ls > 255 || (long)g.N * g.T * g.H * g.W * g.C * 2 > (1L << 30) ||
      (long)Cout * g.Kp * 2 > 0x7fffffffL)
    return 0;
  if ((long)((128 + g.Wo - 2) / g.Wo + 1) * Ls > fr::Cfg<128>::SQ) return 0;
  const long t128 = (long)((M + 127) / 128) * (Cout / fr::TN);
  if (t128 >= 256) return 0;
  const int nks = g.kt * g.kh * (g.C / 64);
  const int s = (int)std::min<long>(4, (512 + t128 - 1) / t128);
  return s >= 2 && nks >= 2 * s ? s : 0;
}
extern "C" long cmhar_conv3d_fwd_split_ws(const int* dims, int Cout) {
  const Geom g = make_geom(dims);
  const int s = fwd_split_count(g, Cout);
  return s ? (long)s * g.N * g.To * g.Ho * g.Wo * Cout : 0;
}
extern "C" int cmhar_conv3d_fwd_split(const int* dims, int Cout, const void* x, const void* w, const void* res,
                                      void* z, float* ws, hipStream_t stream) {
  const Geom g = make_geom(dims);
  const int s = fwd_split_count(g, Cout);
  if (!s || !ws) return -1;
  const int M = g.N * g.To * g.Ho * g.Wo;
  int kps;
  if (ig_split_count(g, Cout, kps)) {
    if (fwd_plan(g, Cout) == 4)
      conv3d_fwd_igemm<2, true><<<dim3((M + 127) / 128, s), 256, 0, stream>>>(
          g, M, Cout, (const bf16*)x, (const bf16*)w, nullptr, nullptr, nullptr, kps, ws);
    else
      conv3d_fwd_igemm<4, true><<<dim3(((M + 127) / 128) * ((Cout + 127) / 128), s), 256, 0, stream>>>(
          g, M, Cout, (const bf16*)x, (const bf16*)w, nullptr, nullptr, nullptr, kps, ws);
    conv_split_reduce<<<grid_for((long)M * Cout / 8), 256, 0, stream>>>(M, Cout, s, ws, (const bf16*)res, (bf16*)z);
    CMHAR_CHECK_LAUNCH();
    return 0;
  }
  const int Ls = (g.Wo - 1) * g.sw + g.kw;
  const int t128 = ((M + 127) / 128) * (Cout / fr::TN);
  conv3d_fwd_rows<128><<<dim3(t128, s), 256, 0, stream>>>(g, M, Cout, Ls, (const bf16*)x, (const bf16*)w, nullptr,
                                                         nullptr, nullptr, ws);
  conv_split_reduce<<<grid_for((long)M * Cout / 8), 256, 0, stream>>>(M, Cout, s, ws, (const bf16*)res, (bf16*)z);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Launch plan of cmhar_conv3d_fwd (exported as cmhar_conv3d_fwd_plan so tests pin the kernel a geometry takes):
// 1 = nine-tap conv3d_fwd_rows3 (Cout = 64, 3x3 taps at unit H/W stride), 2 = row-slab conv3d_fwd_rows<128>,
// 3 = row-slab conv3d_fwd_rows<256>, 4 = generic conv3d_fwd_igemm 128x64, 5 = generic conv3d_fwd_igemm 128x128;
// -1 = not an implicit-GEMM geometry.  (The split-K plan is the caller's choice: cmhar_conv3d_fwd_split_ws > 0.)
// CMHAR_FWD_ROWS=0: the generic gather kernel instead of the row-slab ones (A/B runs).
static int fwd_plan(const Geom& g, int Cout) {
  if (!igemm_ok(g, Cout)) return -1;
  Fwd3Plan p3;
  if (fwd3_plan(g, Cout, p3)) return 1;
  static const bool rows_on = [] {
    const char* v = getenv("CMHAR_FWD_ROWS");
    return !(v && v[0] == '0');
  }();
  const int M = g.N * g.To * g.Ho * g.Wo;
  const int Ls = (g.Wo - 1) * g.sw + g.kw;
  auto fits = [&](int tm, int sq) { return (long)((tm + g.Wo - 2) / g.Wo + 1) * Ls <= sq; };   // rows a tile touches
  if (rows_on && g.kw == 3 && Cout % fr::TN == 0 && g.Wo <= 255 && Ls <= 255 &&
      (long)g.N * g.T * g.H * g.W * g.C * 2 <= (1L << 30) && (long)Cout * g.Kp * 2 <= 0x7fffffffL) {   // 32-bit offsets
    // 256-row tiles while they give every CU a workgroup, else 128-row tiles (R3D-18 layer 4: 268 -> 164 us; layer 3
    // at 392 256-row tiles measured 167 vs 199 us, so it keeps them)
    const long t256 = (long)((M + 255) / 256) * (Cout / fr::TN);
    const bool small = t256 < 256 && fits(128, fr::Cfg<128>::SQ);
    if (small) return 2;
    if (fits(256, fr::Cfg<256>::SQ)) return 3;
  }
  // Cout <= 64: 128x64 tiles (a 128-wide tile would leave half its MFMA work on padding columns)
  return Cout <= 64 ? 4 : 5;
}
extern "C" int cmhar_conv3d_fwd_plan(const int* dims, int Cout) { return fwd_plan(make_geom(dims), Cout); }

extern "C" int cmhar_conv3d_fwd(const int* dims, int Cout, const void* x, const void* w, const void* res, void* z,
                                float* tile_stats, hipStream_t stream) {
  const Geom g = make_geom(dims);
  const int plan = fwd_plan(g, Cout);
  if (plan < 0) return -1;
  const int M = g.N * g.To * g.Ho * g.Wo;
  const int Ls = (g.Wo - 1) * g.sw + g.kw;
  switch (plan) {
    case 1: {
      Fwd3Plan p3;
      fwd3_plan(g, Cout, p3);
      static const bool swz = [] {   // CMHAR_ROWS3_SWZ=0: the padded 144-B LDS rows (A/B runs)
        const char* v = getenv("CMHAR_ROWS3_SWZ");
        return !(v && v[0] == '0');
      }();
      if (swz)
        conv3d_fwd_rows3<true><<<p3.ntile * (Cout / fr3::TN), 256, 0, stream>>>(
            g, Cout, p3.R, p3.Ls, p3.cpf, (const bf16*)x, (const bf16*)w, (const bf16*)res, (bf16*)z, tile_stats);
      else
        conv3d_fwd_rows3<false><<<p3.ntile * (Cout / fr3::TN), 256, 0, stream>>>(
            g, Cout, p3.R, p3.Ls, p3.cpf, (const bf16*)x, (const bf16*)w, (const bf16*)res, (bf16*)z, tile_stats);
      break;
    }
    case 2:
      conv3d_fwd_rows<128><<<((M + 127) / 128) * (Cout / fr::TN), 256, 0, stream>>>(
          g, M, Cout, Ls, (const bf16*)x, (const bf16*)w, (const bf16*)res, (bf16*)z, tile_stats);
      break;
    case 3:
      conv3d_fwd_rows<256><<<((M + 255) / 256) * (Cout / fr::TN), 256, 0, stream>>>(
          g, M, Cout, Ls, (const bf16*)x, (const bf16*)w, (const bf16*)res, (bf16*)z, tile_stats);
      break;
    default: {
      // 32-bit buffer offsets when x and the weights are under 2 GiB
      const bool buf = (long)g.N * g.T * g.H * g.W * g.C * 2 <= 0x7fffffffL && (long)Cout * g.Kp * 2 <= 0x7fffffffL;
#define IG(JN, BUF, GRID)                                                                                        \
  conv3d_fwd_igemm<JN, BUF><<<GRID, 256, 0, stream>>>(g, M, Cout, (const bf16*)x, (const bf16*)w, (const bf16*)res, \
                                                      (bf16*)z, tile_stats, g.K / ig::BK, nullptr)
      if (plan == 4) {
        if (buf) IG(2, true, (M + 127) / 128);
        else IG(2, false, (M + 127) / 128);
      } else {
        if (buf) IG(4, true, ((M + 127) / 128) * ((Cout + 127) / 128));
        else IG(4, false, ((M + 127) / 128) * ((Cout + 127) / 128));
      }
#undef IG
    }
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// ---- implicit stem entry points (bf16, C <= 4, kw <= 8, w-stride 2, Cout = 64) ----
struct StemPlan { int R, cpf, ntile; };
static bool stem_plan(const Geom& g, int Cout, StemPlan& p) {
  if (!geom_ok(g) || !(g.C <= 4 && g.kw <= 8 && g.sw == 2 && g.kh <= stm::KHMAX) || Cout != 64) return false;
  // staged positions: every window column a fragment reads, iw = 0..7 (weights zero past kw), all written (zeros)
  if ((g.Wo - 1) * g.sw + 8 > (stm::RB - 16) / 8 || g.Wo > 256) return false;
  if ((long)g.N * g.T * g.H * g.W * g.C >= (1L << 31)) return false;
  p.R = min(256 / g.Wo, g.Ho);
  while (p.R > 1 && (p.R - 1) * g.sh + g.kh > stm::UMAX) --p.R;
  if ((p.R - 1) * g.sh + g.kh > stm::UMAX) return false;
  p.cpf = (g.Ho + p.R - 1) / p.R;
  p.ntile = g.N * g.To * p.cpf;
  return true;
}
extern "C" int cmhar_conv3d_stem_tiles(const int* dims, int Cout) {
  StemPlan p;
  return stem_plan(make_geom(dims), Cout, p) ? p.ntile : -1;
}
extern "C" long cmhar_conv3d_stem_stats_floats(const int* dims, int Cout) {
  const int nt = cmhar_conv3d_stem_tiles(dims, Cout);
  if (nt <= 0) return -1;
  const int ng = (nt + BN_TG - 1) / BN_TG;
  return 2L * (nt + ng) * Cout + nt + ng;
}
extern "C" int cmhar_conv_pack_stem(int Cout, int C, int kt, int kh, int kw, const float* w, void* out,
                                    hipStream_t stream) {
  if (Cout <= 0 || C <= 0 || C > 4 || kt <= 0 || kh <= 0 || kw <= 0 || kw > 8 || !w || !out) return -1;
  const int n = Cout * kt * kh * 32;
  stem_pack_kernel<<<cdiv(n, 256), 256, 0, stream>>>(Cout, C, kt, kh, kw, w, (bf16*)out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
extern "C" int cmhar_conv3d_stem_fwd(const int* dims, int Cout, const void* x, const void* w4, void* z,
                                     float* tile_stats, hipStream_t stream) {
  const Geom g = make_geom(dims);
  StemPlan p;
  if (!stem_plan(g, Cout, p)) return -1;
  conv3d_stem_fwd<<<p.ntile, 256, 0, stream>>>(g, p.R, p.cpf, (const bf16*)x, (const bf16*)w4, (bf16*)z, tile_stats);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
static int stem_splits(const Geom& g, const StemPlan& p, int& tps) {
  // at most 512 workgroups (rounded up, R3D-18's kt = 3 stem gave 513)
  static const int wgs = [] {   // CMHAR_STEM_WGS: target workgroups (A/B runs)
    const char* v = getenv("CMHAR_STEM_WGS");
    return v ? max(1, atoi(v)) : 512;
  }();
  int s = max(1, min(wgs / g.kt, p.ntile / 8));
  tps = (p.ntile + s - 1) / s;
  return (p.ntile + tps - 1) / tps;
}
extern "C" long cmhar_conv3d_stem_wgrad_ws(const int* dims, int Cout) {
  const Geom g = make_geom(dims);
  StemPlan p;
  if (!stem_plan(g, Cout, p)) return -1;
  int tps;
  const int s = stem_splits(g, p, tps);
  return (long)s * Cout * g.kt * g.kh * 32;
}
extern "C" int cmhar_conv3d_stem_wgrad(const int* dims, int Cout, const void* x, const void* dz, float* dw4, float* ws,
                                       hipStream_t stream) {
  const Geom g = make_geom(dims);
  StemPlan p;
  if (!stem_plan(g, Cout, p) || !ws || !dw4) return -1;
  int tps;
  const int s = stem_splits(g, p, tps);
  conv3d_stem_wgrad<<<dim3(g.kt, s), 64 * stm::KHMAX, 0, stream>>>(g, p.R, p.cpf, p.ntile, tps, (const bf16*)x,
                                                                  (const bf16*)dz, ws);
  const long slab = (long)Cout * g.kt * g.kh * 32, n4 = slab / 4;
  conv3d_wgrad_reduce<<<grid_for(n4), 256, 0, stream>>>(n4, s, slab, ws, dw4);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Split of the M contraction: ~2048 workgroups (8 per CU), slices of >= 512 rows (multiples of 64).  Measured on the
// R3D-18 step (tools/bench_r3d.py, ms/step): 256 WGs 46.5, 512 44.3, 1024 41.1, 2048 39.8, 4096 39.8, 8192 40.7 —
// short slices keep each XCD's gathered input window inside its L2.
static int wgrad_splits(const Geom& g, int Cout, int& mlen) {
  const int M = g.N * g.To * g.Ho * g.Wo;
  const int tiles = ((Cout + 127) / 128) * ((g.K + 127) / 128);
  static const int wgs = [] {   // CMHAR_WGRAD_IG_WGS: target workgroups (A/B runs)
    const char* v = getenv("CMHAR_WGRAD_IG_WGS");
    return v ? max(1, atoi(v)) : 2048;
  }();
  int s = max(1, wgs / tiles);   // whole rounds: rounding up can leave a last round of a few workgroups
  const int smax = (M + 511) / 512;
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  mlen = ((M + s - 1) / s + 63) / 64 * 64;
  return (M + mlen - 1) / mlen;
}

// Row-slab weight-gradient plan (conv3d_wgrad_rows): kw = 3, whole output rows of <= 64 positions per chunk, the
// chunk's input slab within MAXQ rows, Cout a multiple of 64.  Splits of the output-row chunks give ~2048 workgroups
// (>= 4 chunks each); every split writes a full [Cout][K] partial (the kernel covers all K columns of its tiles).
struct RowsPlan { int R, Ls, rows, cps, splits, cot, grp, cpf, nchunk, cs; };
// channels per workgroup of the nine-tap weight gradient (wr3::C3): CMHAR_WGRAD3_CS=32 / 64 overrides the default
#ifndef CMHAR_WGRAD3_CS_DEFAULT
#define CMHAR_WGRAD3_CS_DEFAULT 64
#endif
static int wgrad3_cs() {
  static const int v = [] {
    const char* e = getenv("CMHAR_WGRAD3_CS");
    const int c = e ? atoi(e) : CMHAR_WGRAD3_CS_DEFAULT;
    return c == 32 ? 32 : 64;
  }();
  return v;
}
static bool rows_plan(const Geom& g, int Cout, RowsPlan& p) {
  static const bool on = [] {
    const char* v = getenv("CMHAR_WGRAD_ROWS");
    return !(v && v[0] == '0');
  }();
  if (!on || g.kw != 3 || g.Wo > wr::SLOTS || Cout % 64 || g.C % 64) return false;
  // CMHAR_WGRAD_ROWS3=0: one-tap-row kernel for every shape; 1: nine-tap kernel for Cout = 64 only; 2 (default): also
  // on 64-wide Cout slices of wider convs.  Measured slower there before the buffer-resource loads (R3D-18 layer 2
  // 295.1 -> 311.0 us); with them faster (layer 2 278.7 -> 232.6 us, layer 3 143.3 -> 127.6, step 2198 -> 2221 clips/s,
  // tools/gpu_r05_envab.sh): the nine-tap kernel's longer K per staged chunk beats the 128-wide tiles' slab reuse
  static const int nine = [] {
    const char* v = getenv("CMHAR_WGRAD_ROWS3");
    return v && (v[0] == '0' || v[0] == '1') ? v[0] - '0' : 2;
  }();
  if (nine && (nine == 2 || Cout == 64) && g.kh == 3 && g.sh == 1 && g.sw == 1) {
    // chunks of R output rows of one frame, balanced over the frame (as the nine-tap forward's tiles)
    const int r0 = min(wr3::SLOTS / g.Wo, g.Ho);
    const int cpf = (g.Ho + r0 - 1) / r0, R = (g.Ho + cpf - 1) / cpf;
    const int Ls3 = g.Wo - 1 + g.kw;
    // (and >= 3/4 of the 256 slots used: layer 4's 7 x 7 frames keep the one-tap-row kernel); x and dz within 1 GiB
    // (32-bit buffer offsets)
    if ((R + 2) * Ls3 <= wr3::SQ && (cpf - 1) * R < g.Ho && 4 * R * g.Wo >= 3 * wr3::SLOTS &&
        (long)g.N * g.T * g.H * g.W * g.C * 2 <= (1L << 30) && (long)g.N * g.To * g.Ho * g.Wo * Cout * 2 <= (1L << 30)) {
      p.grp = 9;
      p.cot = 64;
      p.cs = wgrad3_cs();
      p.R = R;
      p.Ls = Ls3;
      p.cpf = cpf;
      p.nchunk = g.N * g.To * p.cpf;
      const int tiles = g.kt * (g.C / p.cs) * (Cout / 64);
      // one 12-wave workgroup per CU (CS = 32: two 6-wave ones): one full round (rounding the split count up gave R3D-18 layer 1 513
      // workgroups: a third round of one; 512 = two rounds wrote twice the split partials — layer 1 382.1 -> 358.6 us,
      // layer 2 209.0 -> 199.5, layer 3 120.2 -> 110.4 at 256, step 2263 -> 2294 clips/s; 768 / 1024: 2189 / 2188),
      // >= 4 chunks each, <= ~80 MB of split partials
      static const int wgs = [] {   // CMHAR_WGRAD3_WGS: target workgroups (A/B runs)
        const char* v = getenv("CMHAR_WGRAD3_WGS");
        return v ? max(1, atoi(v)) : 256;
      }();
      int s = max(1, (p.cs == 64 ? wgs : 2 * wgs) / tiles);
      s = min(s, (int)((80L << 20) / ((long)Cout * g.K * 4)));
      s = max(1, min(s, p.nchunk / 4));
      p.cps = (p.nchunk + s - 1) / s;
      p.splits = (p.nchunk + p.cps - 1) / p.cps;
      p.rows = g.N * g.To * g.Ho;
      return true;
    }
  }
  p.cs = 64;
  p.R = wr::SLOTS / g.Wo;
  p.Ls = (g.Wo - 1) * g.sw + g.kw;
  if (p.R * p.Ls > wr::MAXQ) return false;
  // 32-bit buffer offsets of x and dz
  if ((long)g.N * g.T * g.H * g.W * g.C * 2 > (1L << 30) || (long)g.N * g.To * g.Ho * g.Wo * Cout * 2 > (1L << 30))
    return false;
  p.rows = g.N * g.To * g.Ho;
  p.cot = Cout % 128 == 0 ? 128 : 64;
  // Cout = 64: three kh taps per workgroup when their slabs fit 64 rows each
  // one kh tap per workgroup: three (the whole kh column, 576 dW columns per staged dz chunk) measured 4 % slower on
  // the R3D-18 step — one workgroup per CU at 213 VGPRs, and a third of the workgroups to hide the gather latency
  p.grp = 1;
  const int nchunk = (p.rows + p.R - 1) / p.R;
  const int tiles = g.kt * (g.kh / p.grp) * (g.C / 64) * (Cout / p.cot);
  // at most ~2048 workgroups, >= 8 chunks each, and at most ~56 MB of fp32 partials (every split adds a Cout x K
  // slab that is written here and read back by the reduce: at 2048 workgroups that was ~200 MB per conv, 1.7 ms per
  // step); within that, the split count with the least time ∝ rounds of the 512 workgroup slots x chunks per split
  // (whole rounds: R3D-18 layer 3 takes 7 splits = 504 workgroups, not 6 = 432)
  static const int wgs = [] {   // CMHAR_WGRAD_ROWS_WGS: target workgroups (A/B runs)
    const char* v = getenv("CMHAR_WGRAD_ROWS_WGS");
    return v ? max(1, atoi(v)) : 2048;
  }();
  const int smax = max(1, min(min(wgs / tiles, (int)((56L << 20) / ((long)Cout * g.K * 4))), nchunk / 8));
  long best = -1;
  for (int c = 1; c <= smax; ++c) {
    const int cps = (nchunk + c - 1) / c, sp = (nchunk + cps - 1) / cps;
    const long t = (long)((tiles * sp + 511) / 512) * cps;
    if (best < 0 || t < best) { best = t; p.cps = cps; p.splits = sp; }
  }
  return true;
}

// Launch plan of cmhar_conv3d_wgrad (exported for tests): 1 = nine-tap conv3d_wgrad_rows3, 2 = row-slab
// conv3d_wgrad_rows with 128-wide Cout tiles, 3 = the same with 64-wide tiles, 4 = generic conv3d_wgrad_igemm; each
// followed by conv3d_wgrad_reduce when cmhar_conv3d_wgrad_ws > 0 (split partials); -1 = not implicit-GEMM.
extern "C" int cmhar_conv3d_wgrad_plan(const int* dims, int Cout) {
  const Geom g = make_geom(dims);
  if (!igemm_ok(g, Cout)) return -1;
  RowsPlan rp;
  if (rows_plan(g, Cout, rp)) return rp.grp == 9 ? 1 : rp.cot == 128 ? 2 : 3;
  return 4;
}

extern "C" long cmhar_conv3d_wgrad_ws(const int* dims, int Cout) {
  const Geom g = make_geom(dims);
  if (!igemm_ok(g, Cout)) return -1;
  RowsPlan rp;
  if (rows_plan(g, Cout, rp)) return rp.splits > 1 ? (long)rp.splits * Cout * g.K : 0;
  int mlen;
  const int s = wgrad_splits(g, Cout, mlen);
  return s > 1 ? (long)s * Cout * g.K : 0;
}

extern "C" int cmhar_conv3d_wgrad(const int* dims, int Cout, const void* x, const void* dz, float* dw, float* ws,
                                  hipStream_t stream) {
  const Geom g = make_geom(dims);
  if (!igemm_ok(g, Cout)) return -1;
  const int M = g.N * g.To * g.Ho * g.Wo;
  RowsPlan rp;
  if (rows_plan(g, Cout, rp)) {
    if (rp.splits > 1 && !ws) return -2;
    float* dst = rp.splits > 1 ? ws : dw;
    if (rp.grp == 9) {
      const dim3 grid3(g.kt * (g.C / rp.cs) * (Cout / 64), rp.splits);
      if (rp.cs == 32)
        conv3d_wgrad_rows3<32><<<grid3, wr3::C3<32>::NT, 0, stream>>>(g, Cout, rp.R, rp.Ls, rp.cpf, rp.nchunk, rp.cps,
                                                                      (const bf16*)x, (const bf16*)dz, dst);
      else
        conv3d_wgrad_rows3<64><<<grid3, wr3::C3<64>::NT, 0, stream>>>(g, Cout, rp.R, rp.Ls, rp.cpf, rp.nchunk, rp.cps,
                                                                      (const bf16*)x, (const bf16*)dz, dst);
      if (rp.splits > 1) {
        const long slab = (long)Cout * g.K, n4 = slab / 4;
        conv3d_wgrad_reduce<<<grid_for(n4), 256, 0, stream>>>(n4, rp.splits, slab, ws, dw);
      }
      CMHAR_CHECK_LAUNCH();
      return 0;
    }
    const int tiles = g.kt * (g.kh / rp.grp) * (g.C / 64) * (Cout / rp.cot);
    const dim3 grid(tiles, rp.splits);
#define WR(COT, G, SQ, NW)                                                                                       \
  conv3d_wgrad_rows<COT, G, SQ, NW><<<grid, 64 * NW, 0, stream>>>(g, Cout, rp.R, rp.Ls, rp.rows, rp.cps,          \
                                                                  (const bf16*)x, (const bf16*)dz, dst)
    if (rp.cot == 128) WR(128, 1, 136, 4);
    else WR(64, 1, 136, 4);
#undef WR
    if (rp.splits > 1) {
      const long slab = (long)Cout * g.K, n4 = slab / 4;
      conv3d_wgrad_reduce<<<grid_for(n4), 256, 0, stream>>>(n4, rp.splits, slab, ws, dw);
    }
    CMHAR_CHECK_LAUNCH();
    return 0;
  }
  int mlen;
  const int s = wgrad_splits(g, Cout, mlen);
  if (s > 1 && !ws) return -2;
  const int tiles = ((Cout + 127) / 128) * ((g.K + 127) / 128);
  dim3 grid(tiles, s);
  conv3d_wgrad_igemm<<<grid, 256, 0, stream>>>(g, M, Cout, mlen, (const bf16*)x, (const bf16*)dz, s > 1 ? ws : dw);
  if (s > 1) {
    const long slab = (long)Cout * g.K, n4 = slab / 4;
    conv3d_wgrad_reduce<<<grid_for(n4), 256, 0, stream>>>(n4, s, slab, ws, dw);
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}
