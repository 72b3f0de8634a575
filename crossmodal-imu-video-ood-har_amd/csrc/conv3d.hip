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

// 8-element vector access (16 B for bf16, 32 B for fp32); every call site is 8-element aligned (C % 8 == 0).
template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    const bf16x8 r = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)r[j];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j];
    *(bf16x8*)p = r;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const floatx4 a = *(const floatx4*)p, b = *(const floatx4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    floatx4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    *(floatx4*)p = a;
    *(floatx4*)(p + 4) = b;
  }
};
template <typename T, int V> __device__ __forceinline__ void vload(const T* p, float* v) {
  if constexpr (V == 8) Vec8<T>::load(p, v);
  else for (int j = 0; j < V; ++j) v[j] = to_f<T>(p[j]);
}
template <typename T, int V> __device__ __forceinline__ void vstore(T* p, const float* v) {
  if constexpr (V == 8) Vec8<T>::store(p, v);
  else for (int j = 0; j < V; ++j) p[j] = from_f<T>(v[j]);
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

// Few input channels (the stem: C = 3): one thread per (row, it, ih) copies the kw·C elements of that tap row,
// which are contiguous in both the NDHWC input and the column (clipped at the W padding).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col3d_seg_kernel(Geom g, int M, const TI* __restrict__ x,
                                                           TO* __restrict__ col) {
  const int segs = g.kt * g.kh, seglen = g.kw * g.C;
  const long total = (long)M * segs;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / segs), sg = (int)(i - (long)row * segs);
    const int it = sg / g.kh, ih = sg - it * g.kh;
    int r = row;
    const int wo = r % g.Wo; r /= g.Wo;
    const int ho = r % g.Ho; r /= g.Ho;
    const int to = r % g.To;
    const int n = r / g.To;
    const int ti = to * g.st - g.pt + it, hi = ho * g.sh - g.ph + ih, w0 = wo * g.sw - g.pw;
    TO* dst = col + (long)row * g.Kp + sg * seglen;
    const bool rowok = ti >= 0 && ti < g.T && hi >= 0 && hi < g.H;
    const TI* src = x + ((((long)n * g.T + (rowok ? ti : 0)) * g.H + (rowok ? hi : 0)) * g.W) * g.C;
    for (int e = 0; e < seglen; ++e) {
      const int wi = w0 + e / g.C;
      float v = 0.f;
      if (rowok && wi >= 0 && wi < g.W) v = to_f<TI>(src[(long)wi * g.C + e % g.C]);
      dst[e] = from_f<TO>(v);
    }
    if (sg == segs - 1)
      for (int k = g.K; k < g.Kp; ++k) col[(long)row * g.Kp + k] = from_f<TO>(0.f);
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

// ---- BatchNorm over the [M, C] channels-last view ----------------------------------------------------------------
// Column partial sums over a chunk of rows: each thread reads 8 consecutive channels of a row (one 16-B bf16
// vector), TPR = C/8 threads cover a row and the block's RPI = 256/TPR row slots are combined in a fixed order.
// mode 0: Σx; mode 1: Σ(x−mean)²; mode 2: Σg, Σg·x̂ with g = dy·[y > 0 if relu].  part: [2][nchunk][C].
template <typename T>
__global__ __launch_bounds__(256) void bn_cl_partial(int mode, int M, int C, int rows_per_chunk,
                                                     const T* __restrict__ x, const T* __restrict__ y,
                                                     const T* __restrict__ dy, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, int relu,
                                                     float* __restrict__ part) {
  __shared__ float s0[256][9], s1[256][9];
  const int tid = threadIdx.x;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int slot = tid / TPR, c0 = (tid % TPR) * 8;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(r0 + rows_per_chunk, M);
  float mu[8], rs[8], a0[8], a1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mode ? mean[c0 + j] : 0.f;
    rs[j] = mode == 2 ? rstd[c0 + j] : 0.f;
    a0[j] = a1[j] = 0.f;
  }
  for (int r = r0 + slot; r < r1; r += RPI) {
    const long off = (long)r * C + c0;
    float v[8], gv[8], yv[8];
    Vec8<T>::load(x + off, v);
    if (mode == 2) {
      Vec8<T>::load(dy + off, gv);
      if (relu) Vec8<T>::load(y + off, yv);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (mode == 0) {
        a0[j] += v[j];
      } else if (mode == 1) {
        const float d = v[j] - mu[j];
        a0[j] = fmaf(d, d, a0[j]);
      } else {
        const float gj = relu && yv[j] <= 0.f ? 0.f : gv[j];
        a0[j] += gj;
        a1[j] = fmaf(gj, (v[j] - mu[j]) * rs[j], a1[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { s0[tid][j] = a0[j]; s1[tid][j] = a1[j]; }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float b0 = 0.f, b1 = 0.f;
    for (int sl = 0; sl < RPI; ++sl) { b0 += s0[sl * TPR + c / 8][c % 8]; b1 += s1[sl * TPR + c / 8][c % 8]; }
    part[(long)blockIdx.x * C + c] = b0;
    if (mode == 2) part[((long)gridDim.x + blockIdx.x) * C + c] = b1;
  }
}

// Combine the chunk partials (64 columns per block, 4 chunk slots, fixed order) and finish the statistic.
// mode 0: mean;  mode 1: rstd (+ running stats, num_batches_tracked);  mode 2: db = Σg, dw = Σg·x̂.
__global__ __launch_bounds__(256) void bn_cl_final(int mode, long M, int C, int nchunk, const float* __restrict__ part,
                                                   float* __restrict__ mean, float* __restrict__ rstd,
                                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                                   long long* __restrict__ nbt, float momentum, float eps,
                                                   float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float s0[256], s1[256];
  const int tid = threadIdx.x, cl = tid & 63, slot = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a0 = 0.f, a1 = 0.f;
  if (c < C)
    for (int k = slot; k < nchunk; k += 4) {
      a0 += part[(long)k * C + c];
      if (mode == 2) a1 += part[((long)nchunk + k) * C + c];
    }
  s0[tid] = a0;
  s1[tid] = a1;
  __syncthreads();
  if (slot || c >= C) return;
  const float b0 = s0[cl] + s0[64 + cl] + s0[128 + cl] + s0[192 + cl];
  const float b1 = s1[cl] + s1[64 + cl] + s1[128 + cl] + s1[192 + cl];
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

__global__ void bn_cl_eval_stats(int C, const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                 float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) { mean[c] = rmean[c]; rstd[c] = rsqrtf(rvar[c] + eps); }
}

// y = relu?((x − mean)·rstd·w + b + res), 8 channels per thread
template <typename T>
__global__ __launch_bounds__(256) void bn_cl_apply(unsigned nvec, int C, const T* __restrict__ x,
                                                   const T* __restrict__ res, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* __restrict__ w,
                                                   const float* __restrict__ b, int relu, T* __restrict__ y) {
  const unsigned cv = C / 8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * 8;
    const long off = (long)i * 8;
    float v[8], rv[8];
    Vec8<T>::load(x + off, v);
    if (res) Vec8<T>::load(res + off, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      v[j] = fmaf((v[j] - mean[c]) * rstd[c], w[c], b[c]);
      if (res) v[j] += rv[j];
      if (relu) v[j] = fmaxf(v[j], 0.f);
    }
    Vec8<T>::store(y + off, v);
  }
}

// g = dy·[y > 0];  dres = g (optional);  dx = w·rstd·(g − Σg/M − x̂·Σgx̂/M) (training) or w·rstd·g (eval).
template <typename T>
__global__ __launch_bounds__(256) void bn_cl_bwd_apply(unsigned nvec, int M, int C, const T* __restrict__ x,
                                                       const T* __restrict__ y, const T* __restrict__ dy,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ w, const float* __restrict__ dw,
                                                       const float* __restrict__ db, int training, int relu,
                                                       T* __restrict__ dx, T* __restrict__ dres) {
  const float inv = 1.f / (float)M;
  const unsigned cv = C / 8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * 8;
    const long off = (long)i * 8;
    float gv[8], yv[8], xv[8], out[8];
    Vec8<T>::load(dy + off, gv);
    if (relu) Vec8<T>::load(y + off, yv);
    if (training) Vec8<T>::load(x + off, xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      if (relu && yv[j] <= 0.f) gv[j] = 0.f;
      const float rs = rstd[c];
      if (training) {
        const float xh = (xv[j] - mean[c]) * rs;
        out[j] = w[c] * rs * (gv[j] - db[c] * inv - xh * dw[c] * inv);
      } else {
        out[j] = w[c] * rs * gv[j];
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
    for (long s = slot; s < S; s += RPI) a += to_f<T>(x[((long)n * S + s) * C + c0 + cc]);
    sh[tid] = a;
    __syncthreads();
    if (slot == 0) {
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

inline int grid_for(long work) {
  const long b = (work + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

inline bool bn_channels_ok(int C) { return C >= 8 && C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0; }

inline int bn_chunks(long M) {   // ≤ 512 chunks of ≥ 512 rows: enough blocks to stream M·C, few partials to combine
  const long c = (M + 511) / 512;
  return (int)(c < 512 ? (c > 0 ? c : 1) : 512);
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
  const bool seg = false;   // measured: the coalesced per-element row kernel beats the per-thread segment copy
  const int kv = vec ? g.Kp / 8 : g.Kp;
  int tpr = 1;
  while (tpr < kv && tpr < 256) tpr <<= 1;
  const int rows_grid = grid_for((long)M * tpr);
  const int seg_grid = grid_for((long)M * g.kt * g.kh);
#define IM2COL(TI, TO)                                                                                          \
  do {                                                                                                          \
    if (vec) im2col3d_kernel<TI, TO, 8><<<rows_grid, 256, 0, stream>>>(g, M, tpr, (const TI*)x, (TO*)col);     \
    else if (seg) im2col3d_seg_kernel<TI, TO><<<seg_grid, 256, 0, stream>>>(g, M, (const TI*)x, (TO*)col);    \
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
  if (dtype == CMHAR_BF16) {
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

extern "C" long cmhar_bn_cl_ws(long M, int C) { return 2L * bn_chunks(M) * C; }

extern "C" int cmhar_bn_cl_fwd(int dtype, long M, int C, const void* x, const void* res, void* y, const float* w,
                               const float* b, float* rmean, float* rvar, float* smean, float* srstd, int training,
                               float momentum, float eps, int relu, long long* num_batches_tracked, float* ws,
                               hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !ws) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 32)) return -2;
  const int nch = bn_chunks(M);
  const int rpc = (int)((M + nch - 1) / nch);
  const int fgrid = (C + 63) / 64;
  if (training) {
    for (int mode = 0; mode < 2; ++mode) {
      if (dtype == CMHAR_BF16)
        bn_cl_partial<bf16><<<nch, 256, 0, stream>>>(mode, (int)M, C, rpc, (const bf16*)x, nullptr, nullptr, smean,
                                                     nullptr, 0, ws);
      else if (dtype == CMHAR_F32)
        bn_cl_partial<float><<<nch, 256, 0, stream>>>(mode, (int)M, C, rpc, (const float*)x, nullptr, nullptr, smean,
                                                      nullptr, 0, ws);
      else return -1;
      bn_cl_final<<<fgrid, 256, 0, stream>>>(mode, M, C, nch, ws, smean, srstd, rmean, rvar, num_batches_tracked,
                                             momentum, eps, nullptr, nullptr);
    }
  } else {
    if (!rmean || !rvar) return -2;
    bn_cl_eval_stats<<<(C + 255) / 256, 256, 0, stream>>>(C, rmean, rvar, eps, smean, srstd);
  }
  const unsigned nvec = (unsigned)(M * C / 8);
  if (dtype == CMHAR_BF16)
    bn_cl_apply<bf16><<<grid_for(nvec), 256, 0, stream>>>(nvec, C, (const bf16*)x, (const bf16*)res, smean, srstd,
                                                           w, b, relu, (bf16*)y);
  else
    bn_cl_apply<float><<<grid_for(nvec), 256, 0, stream>>>(nvec, C, (const float*)x, (const float*)res, smean,
                                                            srstd, w, b, relu, (float*)y);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_bn_cl_bwd(int dtype, long M, int C, const void* x, const void* y, const void* dy,
                               const float* w, const float* smean, const float* srstd, void* dx, void* dres,
                               float* dw, float* db, int training, int relu, float* ws, hipStream_t stream) {
  if (M <= 0 || !bn_channels_ok(C) || !ws || !dw || !db) return -1;
  if (M >= (1L << 31) || M * C / 8 >= (1L << 32)) return -2;
  const int nch = bn_chunks(M);
  const int rpc = (int)((M + nch - 1) / nch);
  if (dtype == CMHAR_BF16)
    bn_cl_partial<bf16><<<nch, 256, 0, stream>>>(2, (int)M, C, rpc, (const bf16*)x, (const bf16*)y, (const bf16*)dy,
                                                 smean, srstd, relu, ws);
  else if (dtype == CMHAR_F32)
    bn_cl_partial<float><<<nch, 256, 0, stream>>>(2, (int)M, C, rpc, (const float*)x, (const float*)y, (const float*)dy,
                                                  smean, srstd, relu, ws);
  else return -1;
  bn_cl_final<<<(C + 63) / 64, 256, 0, stream>>>(2, M, C, nch, ws, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f,
                                                 0.f, dw, db);
  const unsigned nvec = (unsigned)(M * C / 8);
  if (dtype == CMHAR_BF16)
    bn_cl_bwd_apply<bf16><<<grid_for(nvec), 256, 0, stream>>>(nvec, (int)M, C, (const bf16*)x, (const bf16*)y,
                                                               (const bf16*)dy, smean, srstd, w, dw, db, training,
                                                               relu, (bf16*)dx, (bf16*)dres);
  else
    bn_cl_bwd_apply<float><<<grid_for(nvec), 256, 0, stream>>>(nvec, (int)M, C, (const float*)x, (const float*)y,
                                                                (const float*)dy, smean, srstd, w, dw, db, training,
                                                                relu, (float*)dx, (float*)dres);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_avgpool_cl(int dtype, int N, long S, int C, const void* x, float* out, hipStream_t stream) {
  if (N <= 0 || S <= 0 || !bn_channels_ok(C)) return -1;
  const int CB = C < 256 ? C : 256;
  dim3 grid(C / CB, N);
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
