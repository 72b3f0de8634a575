// Per-frame 2-D CNN video backbones of the reference's VideoEncoder (src/models/models.py:163-173, forward :208-216:
// torchvision resnet18 children[:-2] / mobilenet_v2 .features over (B·T, 3, H, W) frames).  Dense convolutions run
// on the conv3d kernels with kt = 1 (implicit GEMM on MFMA / im2col + GEMM, csrc/conv3d.hip); this file holds what
// those networks add, all channels-last NHWC ([frames, H, W, C], 8 consecutive channels per thread = one 16-B bf16
// vector):
//   * MaxPool2d(3, 2, 1) of the ResNet stem: forward keeps the argmax tap (uint8, first maximum in scan order as
//     torch's CPU kernel) and the backward is a GATHER over the ≤ ceil(k/s)² windows covering an input pixel — no
//     atomics, deterministic;
//   * depthwise Conv2d(C, C, k, s, p, groups=C) of MobileNetV2's inverted residuals: forward and input gradient
//     (gather form) are one pass each; the weight gradient Σ_rows dz·x_tap is a two-level fixed-order reduction
//     (per-chunk partial slabs [nchunk][taps][C], then a chunk-ordered sum);
//   * weight packing [Cout, Cin, kt, kh, kw] fp32 → [Cout, Kp] compute dtype in the im2col k order (and the
//     tap-flipped, in/out-transposed form the stride-1 input gradient convolves with) — one launch instead of a
//     chain of torch permute / copy kernels per conv per step.
#include "common.h"

namespace {

inline int grid_for(long work) {
  const long b = (work + 255) / 256;
  return (int)(b < 65536L * 8 ? (b > 0 ? b : 1) : 65536L * 8);
}

struct Pool {
  int N, H, W, C, k, s, p, Ho, Wo;
};

// ---- MaxPool2d ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void maxpool_cl_fwd(Pool g, const T* __restrict__ x, T* __restrict__ y,
                                                      unsigned char* __restrict__ idx) {
  const int cv = g.C / 8;
  // 32-bit index decomposition (host-checked: N·Ho·Wo·C/8 < 2^31): 64-bit division is a long software sequence
  const unsigned total = (unsigned)g.N * g.Ho * g.Wo * cv;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (unsigned)cv) * 8;
    unsigned r = i / (unsigned)cv;
    const int wo = (int)(r % (unsigned)g.Wo); r /= (unsigned)g.Wo;
    const int ho = (int)(r % (unsigned)g.Ho);
    const int n = (int)(r / (unsigned)g.Ho);
    float best[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
    for (int ih = 0; ih < g.k; ++ih) {
      const int h = ho * g.s - g.p + ih;
      if (h < 0 || h >= g.H) continue;
      for (int iw = 0; iw < g.k; ++iw) {
        const int w = wo * g.s - g.p + iw;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<T>::load(x + (((long)n * g.H + h) * g.W + w) * g.C + c0, v);
        const int tap = ih * g.k + iw;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          // torch's rule (max_pool2d CPU/GPU kernels): strict > keeps the first maximum in scan order, and a NaN
          // always wins (each later NaN too), so a NaN in the window propagates with the gradient to the last NaN
          if (v[j] > best[j] || __builtin_isnan(v[j])) { best[j] = v[j]; arg[j] = tap; }
      }
    }
    const size_t o = (size_t)i * 8;
    Vec8<T>::store(y + o, best);
    uint2_t a;
    a[0] = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    a[1] = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *(uint2_t*)(idx + o) = a;
  }
}

// dx[n, h, w, c] = Σ over the windows (ho, wo) that contain (h, w) and whose argmax is that tap of dy[n, ho, wo, c]
template <typename T>
__global__ __launch_bounds__(256) void maxpool_cl_bwd(Pool g, const T* __restrict__ dy,
                                                      const unsigned char* __restrict__ idx, T* __restrict__ dx) {
  const int cv = g.C / 8;
  const unsigned total = (unsigned)g.N * g.H * g.W * cv;     // < 2^31 (host-checked)
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (unsigned)cv) * 8;
    unsigned r = i / (unsigned)cv;
    const int w = (int)(r % (unsigned)g.W); r /= (unsigned)g.W;
    const int h = (int)(r % (unsigned)g.H);
    const int n = (int)(r / (unsigned)g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // windows ho with ho·s − p ≤ h ≤ ho·s − p + k − 1
    const int ho_lo = max(0, (h + g.p - g.k + g.s) / g.s), ho_hi = min(g.Ho - 1, (h + g.p) / g.s);
    const int wo_lo = max(0, (w + g.p - g.k + g.s) / g.s), wo_hi = min(g.Wo - 1, (w + g.p) / g.s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int ih = h + g.p - ho * g.s;
      if (ih < 0 || ih >= g.k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int iw = w + g.p - wo * g.s;
        if (iw < 0 || iw >= g.k) continue;
        const long o = (((long)n * g.Ho + ho) * g.Wo + wo) * g.C + c0;
        const uint2_t a = *(const uint2_t*)(idx + o);
        float v[8];
        Vec8<T>::load(dy + o, v);
        const int tap = ih * g.k + iw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int aj = (int)((a[j >> 2] >> (8 * (j & 3))) & 0xff);
          if (aj == tap) acc[j] += v[j];
        }
      }
    }
    Vec8<T>::store(dx + (size_t)i * 8, acc);
  }
}

// ---- depthwise Conv2d -----------------------------------------------------------------------------------------
// weights: the nn.Conv2d parameter itself, fp32 [C, 1, K, K] (w[c·K² + tap]).  A thread's 8 channels own the
// contiguous run w[c0·K² .. (c0+8)·K²): it is fetched as 2·K² 16-B loads into registers (per element the weights
// compiled to 8·K² scalar loads per 8 outputs — the kernels' bottleneck).  K is a template parameter so every tap
// loop and weight index is static.
template <int K>
__device__ __forceinline__ void load_dw_weights(const float* __restrict__ wt, int c0, float (&wv)[8 * K * K]) {
  const floatx4* src = (const floatx4*)(wt + c0 * K * K);
#pragma unroll
  for (int q = 0; q < 2 * K * K; ++q) {
    const floatx4 t = src[q];
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[4 * q + j] = t[j];
  }
}

// 8 elements of T through a buffer resource, issued (ld) apart from their use (get): the K² taps of an output are
// all in flight together.  An offset with bit 31 set lies past the resource (whose range the launch keeps within
// 2^31 bytes) and reads zero: the padding taps need no branch around their load — a branch per tap made every
// tap's load wait for the previous one — and contribute fmaf(0, w, acc) = acc, the same sum as skipping them.
template <typename T> struct Raw8;
template <> struct Raw8<bf16> {
  uint4_t r;
  __device__ __forceinline__ void ld(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    r = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
  __device__ __forceinline__ void get(float* v) const {
    const bf16x8 b = __builtin_bit_cast(bf16x8, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
  }
};
template <> struct Raw8<float> {
  uint4_t a, b;
  __device__ __forceinline__ void ld(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    a = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    b = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
  }
  __device__ __forceinline__ void get(float* v) const {
    const floatx4 x0 = __builtin_bit_cast(floatx4, a), x1 = __builtin_bit_cast(floatx4, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = x0[j]; v[4 + j] = x1[j]; }
  }
};
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const T* p, long elems) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)min(elems * (long)sizeof(T), 0x7fffffffL),
                                           0x00020000);
}
// byte offset of element e, or past the range when !ok
template <typename T>
__device__ __forceinline__ unsigned buf_off(int e, bool ok) {
  return (unsigned)(e * (int)sizeof(T)) | ((unsigned)!ok << 31);
}
// the buffer form applies when every tensor the kernel reads stays below 2^31 bytes
inline bool dw_buf_ok(long elems, int dtype_bytes) { return elems * dtype_bytes < (1L << 31); }

template <typename T, int K, bool BUF>
__global__ __launch_bounds__(256) void dwconv_cl_fwd(Pool g, const T* __restrict__ x, const float* __restrict__ wt,
                                                     T* __restrict__ z) {
  const int cv = g.C / 8;
  // 32-bit index decomposition (host-checked: N·Ho·Wo·C/8 < 2^31): 64-bit division is a long software sequence
  const unsigned total = (unsigned)g.N * g.Ho * g.Wo * cv;
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(x, (long)g.N * g.H * g.W * g.C);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (unsigned)cv) * 8;
    unsigned r = i / (unsigned)cv;
    const int wo = (int)(r % (unsigned)g.Wo); r /= (unsigned)g.Wo;
    const int ho = (int)(r % (unsigned)g.Ho);
    const int n = (int)(r / (unsigned)g.Ho);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (BUF) {
      Raw8<T> rv[K * K];
#pragma unroll
      for (int t = 0; t < K * K; ++t) {
        const int h = ho * g.s - g.p + t / K, w = wo * g.s - g.p + t % K;
        rv[t].ld(xr, buf_off<T>(((n * g.H + h) * g.W + w) * g.C + c0, h >= 0 && h < g.H && w >= 0 && w < g.W));
      }
      float wv[8 * K * K];
      load_dw_weights<K>(wt, c0, wv);
#pragma unroll
      for (int t = 0; t < K * K; ++t) {
        float v[8];
        rv[t].get(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wv[j * K * K + t], acc[j]);
      }
    } else {
      float wv[8 * K * K];
      load_dw_weights<K>(wt, c0, wv);
      const T* xn = x + (size_t)n * g.H * g.W * g.C + c0;
#pragma unroll
      for (int ih = 0; ih < K; ++ih) {
        const int h = ho * g.s - g.p + ih;
#pragma unroll
        for (int iw = 0; iw < K; ++iw) {
          const int w = wo * g.s - g.p + iw;
          if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
            float v[8];
            Vec8<T>::load(xn + ((size_t)h * g.W + w) * g.C, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wv[j * K * K + ih * K + iw], acc[j]);
          }
        }
      }
    }
    Vec8<T>::store(z + (size_t)i * 8, acc);
  }
}

// dx[n, h, w, c] = Σ_taps dz[n, ho, wo, c] · w[c, tap] over the outputs whose window holds (h, w) at that tap
template <typename T, int K, bool BUF>
__global__ __launch_bounds__(256) void dwconv_cl_dgrad(Pool g, const T* __restrict__ dz, const float* __restrict__ wt,
                                                       T* __restrict__ dx) {
  const int cv = g.C / 8;
  const unsigned total = (unsigned)g.N * g.H * g.W * cv;     // < 2^31 (host-checked)
  const __amdgpu_buffer_rsrc_t dzr = buf_rsrc(dz, (long)g.N * g.Ho * g.Wo * g.C);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (unsigned)cv) * 8;
    unsigned r = i / (unsigned)cv;
    const int w = (int)(r % (unsigned)g.W); r /= (unsigned)g.W;
    const int h = (int)(r % (unsigned)g.H);
    const int n = (int)(r / (unsigned)g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (BUF) {
      Raw8<T> rv[K * K];
#pragma unroll
      for (int t = 0; t < K * K; ++t) {
        const int hh = h + g.p - t / K, ww = w + g.p - t % K, ho = hh / g.s, wo = ww / g.s;
        const bool ok = hh >= 0 && hh % g.s == 0 && ho < g.Ho && ww >= 0 && ww % g.s == 0 && wo < g.Wo;
        rv[t].ld(dzr, buf_off<T>(((n * g.Ho + ho) * g.Wo + wo) * g.C + c0, ok));
      }
      float wv[8 * K * K];
      load_dw_weights<K>(wt, c0, wv);
#pragma unroll
      for (int t = 0; t < K * K; ++t) {
        float v[8];
        rv[t].get(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wv[j * K * K + t], acc[j]);
      }
      Vec8<T>::store(dx + (size_t)i * 8, acc);
      continue;
    }
    float wv[8 * K * K];
    load_dw_weights<K>(wt, c0, wv);
    const T* dzn = dz + (size_t)n * g.Ho * g.Wo * g.C + c0;
#pragma unroll
    for (int ih = 0; ih < K; ++ih) {
      const int hh = h + g.p - ih;
      const int ho = hh / g.s;
#pragma unroll
      for (int iw = 0; iw < K; ++iw) {
        const int ww = w + g.p - iw;
        const int wo = ww / g.s;
        if (hh >= 0 && hh % g.s == 0 && ho < g.Ho && ww >= 0 && ww % g.s == 0 && wo < g.Wo) {
          float v[8];
          Vec8<T>::load(dzn + ((size_t)ho * g.Wo + wo) * g.C, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], wv[j * K * K + ih * K + iw], acc[j]);
        }
      }
    }
    Vec8<T>::store(dx + (size_t)i * 8, acc);
  }
}

// Weight-gradient partials: chunk b of rows_per_chunk output rows, thread = (row slot, 8 channels), K² taps of 8
// accumulators in registers; two rows per iteration so the next row's 1 + K² loads are in flight under the current
// row's FMAs; the block's row slots are combined in a fixed order through LDS one tap at a time.
// part: [nchunk][K²][C].
template <typename T, int K, bool BUF>
__global__ __launch_bounds__(256) void dwconv_cl_wgrad_partial(Pool g, int rows_per_chunk, const T* __restrict__ x,
                                                               const T* __restrict__ dz, float* __restrict__ part) {
  constexpr int KK = K * K;
  __shared__ float sh[256][9];
  const int tid = threadIdx.x;
  const int TPR = g.C / 8, RPI = 256 / TPR;
  const int slot = tid / TPR, c0 = (tid % TPR) * 8;
  const long M = (long)g.N * g.Ho * g.Wo;
  const long r0 = (long)blockIdx.x * rows_per_chunk;
  const long r1 = min(r0 + rows_per_chunk, M);
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(x, (long)g.N * g.H * g.W * g.C);
  float acc[KK][8];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  auto row_acc = [&](long row) __attribute__((always_inline)) {
    unsigned r = (unsigned)row;                                 // M < 2^31 (host-checked)
    const int wo = (int)(r % (unsigned)g.Wo); r /= (unsigned)g.Wo;
    const int ho = (int)(r % (unsigned)g.Ho);
    const int n = (int)(r / (unsigned)g.Ho);
    float gz[8];
    Vec8<T>::load(dz + (size_t)row * g.C + c0, gz);
    if constexpr (BUF) {
      Raw8<T> rv[KK];
#pragma unroll
      for (int t = 0; t < KK; ++t) {
        const int h = ho * g.s - g.p + t / K, w = wo * g.s - g.p + t % K;
        rv[t].ld(xr, buf_off<T>(((n * g.H + h) * g.W + w) * g.C + c0, h >= 0 && h < g.H && w >= 0 && w < g.W));
      }
#pragma unroll
      for (int t = 0; t < KK; ++t) {
        float v[8];
        rv[t].get(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[t][j] = fmaf(gz[j], v[j], acc[t][j]);
      }
      return;
    }
    const T* xn = x + (size_t)n * g.H * g.W * g.C + c0;
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      const int h = ho * g.s - g.p + t / K, w = wo * g.s - g.p + t % K;
      if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
        float v[8];
        Vec8<T>::load(xn + ((size_t)h * g.W + w) * g.C, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[t][j] = fmaf(gz[j], v[j], acc[t][j]);
      }
    }
  };
  if (slot < RPI) {
    long row = r0 + slot;
    for (; row + RPI < r1; row += 2 * RPI) {
      row_acc(row);
      row_acc(row + RPI);
    }
    if (row < r1) row_acc(row);
  }
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[tid][j] = acc[t][j];
    __syncthreads();
    for (int c = tid; c < g.C; c += 256) {
      float b = 0.f;
      for (int sl = 0; sl < RPI; ++sl) b += sh[sl * TPR + c / 8][c % 8];
      part[((long)blockIdx.x * KK + t) * g.C + c] = b;
    }
  }
}

// dw[c, tap] = Σ_chunks part[chunk][tap][c]: a block sums 32 channels (lanes, coalesced 128-B rows of the slab) of one
// tap over 8 chunk slots in a fixed order, then the slots in a fixed order
__global__ __launch_bounds__(256) void dwconv_cl_wgrad_final(int C, int kk, int nchunk, const float* __restrict__ part,
                                                             float* __restrict__ dw) {
  __shared__ float sh[256];
  const int tid = threadIdx.x, cl = tid & 31, slot = tid >> 5;
  const int c = blockIdx.x * 32 + cl, t = blockIdx.y;
  float a = 0.f;
  if (c < C)
    for (int b = slot; b < nchunk; b += 8) a += part[((long)b * kk + t) * C + c];
  sh[tid] = a;
  __syncthreads();
  if (slot == 0 && c < C) {
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) r += sh[k * 32 + cl];
    dw[c * kk + t] = r;
  }
}

inline int dw_chunks(long M) {   // ≤ 2048 chunks of ≥ 256 rows (≥ 8 blocks per CU at production sizes)
  const long c = (M + 255) / 256;
  return (int)(c < 2048 ? (c > 0 ? c : 1) : 2048);
}

// ---- weight packing -------------------------------------------------------------------------------------------
// One pass over the fp32 master w [Cout][Cin][taps] (taps = kt·kh·kw) writes both compute-dtype forms:
//   out  [Cout][Kp]: out[co][tap·Cin + ci] = w[co][ci][tap], zero for k in [K, Kp)      (the im2col k order)
//   outf [Cin][K']:  outf[ci][(taps−1−tap)·Cout + co] = w[co][ci][tap]                  (tap-flipped, transposed:
//                    the weight the stride-1 input gradient convolves dz with)
// A block stages a CO_T × CI_T × taps brick of w in LDS with coalesced reads (for each co the brick is one
// contiguous run of CI_T·taps floats), then writes ci-contiguous segments of `out` and co-contiguous segments of
// `outf` from it.
constexpr int PACK_CO = 32, PACK_LDS = 12288;     // floats (48 KiB)
// i / d for 0 <= i, i·d < 2^32 as one multiply-high (m = ⌈2^32 / d⌉, exact under that bound); the pack's index maps
// had four runtime integer divisions per element and ran the step's 19 packs at ~0.5 TB/s.
struct PackDiv {
  unsigned d, m;
  __device__ __forceinline__ int q(int i) const { return d == 1 ? i : (int)__umulhi((unsigned)i, m); }
};
inline PackDiv pack_div(int d) { return PackDiv{(unsigned)d, d == 1 ? 0u : (unsigned)((0x100000000ull + d - 1) / d)}; }
// V8 (Cin, Cout, Kp and ci_t multiples of 8): each thread gathers 8 channels from the brick and writes them as one
// 16-B vector (2-B scalar stores left the kernel store-issue bound).
template <typename T, bool V8>
__device__ __forceinline__ void conv_pack_block(int bx, int by, float* brick, int Cout, int Cin, int taps, int Kp,
                                                int ci_t, PackDiv d_taps, const float* __restrict__ w,
                                                T* __restrict__ out, T* __restrict__ outf) {
  const int co0 = bx * PACK_CO, ci0 = by * ci_t;
  const int nco = min(PACK_CO, Cout - co0), nci = min(ci_t, Cin - ci0);
  const int run = nci * taps;                      // contiguous floats per co
  const PackDiv d_run{(unsigned)run, run == 1 ? 0u : (unsigned)((0x100000000ull + run - 1) / run)};
  const PackDiv d_nci{(unsigned)nci, nci == 1 ? 0u : (unsigned)((0x100000000ull + nci - 1) / nci)};
  const PackDiv d_nco{(unsigned)nco, nco == 1 ? 0u : (unsigned)((0x100000000ull + nco - 1) / nco)};
  for (int i = threadIdx.x; i < nco * run; i += 256) {
    const int c = d_run.q(i), e = i - c * run;
    brick[c * run + e] = w[((long)(co0 + c) * Cin + ci0) * taps + e];
  }
  __syncthreads();
  if (out && V8) {
    const int n8 = nci >> 3;
    const PackDiv d_n8{(unsigned)n8, n8 == 1 ? 0u : (unsigned)((0x100000000ull + n8 - 1) / n8)};
    for (int i = threadIdx.x; i < nco * taps * n8; i += 256) {       // 8-channel groups, ci fastest
      const int r = d_n8.q(i), g = i - r * n8, c = d_taps.q(r), tap = r - c * taps;
      const float* src = brick + c * run + 8 * g * taps + tap;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[j * taps];
      Vec8<T>::store(out + (long)(co0 + c) * Kp + (long)tap * Cin + ci0 + 8 * g, v);
    }
  } else if (out) {
    for (int i = threadIdx.x; i < nco * taps * nci; i += 256) {      // ci fastest
      const int r = d_nci.q(i), ci = i - r * nci, c = d_taps.q(r), tap = r - c * taps;
      out[(long)(co0 + c) * Kp + (long)tap * Cin + ci0 + ci] = from_f<T>(brick[c * run + ci * taps + tap]);
    }
  }
  if (out) {
    if (by == 0) {                                  // zero padding k in [K, Kp)
      const int K = taps * Cin, pad = Kp - K;
      for (int i = threadIdx.x; i < nco * pad; i += 256)
        out[(long)(co0 + i / pad) * Kp + K + i % pad] = from_f<T>(0.f);
    }
  }
  if (outf && V8) {
    const int n8 = nco >> 3;
    const PackDiv d_n8{(unsigned)n8, n8 == 1 ? 0u : (unsigned)((0x100000000ull + n8 - 1) / n8)};
    for (int i = threadIdx.x; i < nci * taps * n8; i += 256) {       // 8-output groups, co fastest
      const int r = d_n8.q(i), g = i - r * n8, ci = d_taps.q(r), tap = r - ci * taps;
      const float* src = brick + 8 * g * run + ci * taps + tap;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[j * run];
      Vec8<T>::store(outf + (long)(ci0 + ci) * taps * Cout + (long)(taps - 1 - tap) * Cout + co0 + 8 * g, v);
    }
  } else if (outf) {
    for (int i = threadIdx.x; i < nci * taps * nco; i += 256) {      // co fastest
      const int r = d_nco.q(i), c = i - r * nco, ci = d_taps.q(r), tap = r - ci * taps;
      outf[(long)(ci0 + ci) * taps * Cout + (long)(taps - 1 - tap) * Cout + co0 + c] =
          from_f<T>(brick[c * run + ci * taps + tap]);
    }
  }
}

template <typename T, bool V8>
__global__ __launch_bounds__(256) void conv_pack_kernel(int Cout, int Cin, int taps, int Kp, int ci_t, PackDiv d_taps,
                                                        const float* __restrict__ w, T* __restrict__ out,
                                                        T* __restrict__ outf) {
  __shared__ float brick[PACK_LDS];
  conv_pack_block<T, V8>(blockIdx.x, blockIdx.y, brick, Cout, Cin, taps, Kp, ci_t, d_taps, w, out, outf);
}

// All of a network's weight packs in one launch (the per-conv launches were 19 serial small kernels per R3D-18
// step, most of them a few blocks): job k owns the blocks [blk0_k, blk0_{k+1}) of a 1-D grid, laid out as its own
// (gx × gy) pack grid.  Jobs passed by value (≤ PACK_JOBS per launch).
constexpr int PACK_JOBS = 24;
struct PackJob {
  const float* w;
  void* out;
  void* outf;
  int Cout, Cin, taps, Kp, ci_t, gx, blk0, v8;
  PackDiv d_taps;
};
struct PackJobs {
  int n;
  PackJob j[PACK_JOBS];
};
template <typename T>
__global__ __launch_bounds__(256) void conv_pack_multi_kernel(PackJobs jobs) {
  __shared__ float brick[PACK_LDS];
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < jobs.n && b >= jobs.j[k + 1].blk0) ++k;
  const PackJob& J = jobs.j[k];
  const int local = b - J.blk0, bx = local % J.gx, by = local / J.gx;
  if (J.v8)
    conv_pack_block<T, true>(bx, by, brick, J.Cout, J.Cin, J.taps, J.Kp, J.ci_t, J.d_taps, J.w, (T*)J.out,
                             (T*)J.outf);
  else
    conv_pack_block<T, false>(bx, by, brick, J.Cout, J.Cin, J.taps, J.Kp, J.ci_t, J.d_taps, J.w, (T*)J.out,
                              (T*)J.outf);
}

// Weight gradient [Cout][Kp] fp32 in a packed k order → the parameter layout [Cout][Cin][R][kw] (R = kt·kh tap rows):
// source offset co·Kp + r·rs + iw·cs + ci (im2col order: rs = kw·Cin, cs = Cin; implicit stem: rs = 32, cs = 4).  One
// thread per destination element, coalesced writes (replaces the strided-view copy torch's gradient accumulation made).
__global__ __launch_bounds__(256) void conv_grad_unpack_kernel(unsigned n, int Cin, int R, int kw, int Kp, int rs,
                                                               int cs, PackDiv d_kw, PackDiv d_R, PackDiv d_ci,
                                                               const float* __restrict__ src, float* __restrict__ dst) {
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const int t = d_kw.q((int)i), iw = (int)i - t * kw;
    const int t2 = d_R.q(t), r = t - t2 * R;
    const int co = d_ci.q(t2), ci = t2 - co * Cin;
    dst[i] = src[(long)co * Kp + (long)r * rs + iw * cs + ci];
  }
}

Pool make_pool(int N, int H, int W, int C, int k, int s, int p) {
  Pool g{N, H, W, C, k, s, p, 0, 0};
  g.Ho = (H + 2 * p - k) / s + 1;
  g.Wo = (W + 2 * p - k) / s + 1;
  return g;
}

bool pool_ok(const Pool& g) {
  return g.N > 0 && g.H > 0 && g.W > 0 && g.C >= 8 && g.C % 8 == 0 && g.k > 0 && g.k <= 3 &&
         g.s > 0 && g.p >= 0 && 2 * g.p <= g.k && g.Ho > 0 && g.Wo > 0 &&
         (long)g.N * g.H * g.W * (g.C / 8) < (1L << 31) && (long)g.N * g.Ho * g.Wo * (g.C / 8) < (1L << 31) &&
         (long)g.N * g.Ho * g.Wo < (1L << 31);     // (unsigned grid-stride loops: i + stride cannot wrap)
}

}  // namespace

#define DT_SWITCH(dtype, F)                       \
  do {                                            \
    if ((dtype) == CMHAR_BF16) { F(bf16); }       \
    else if ((dtype) == CMHAR_F32) { F(float); }  \
    else return -1;                               \
  } while (0)

extern "C" int cmhar_maxpool2d_cl_fwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x,
                                      void* y, unsigned char* argmax, hipStream_t stream) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g) || !argmax) return -1;
  const long work = (long)N * g.Ho * g.Wo * (C / 8);
#define F(T) maxpool_cl_fwd<T><<<grid_for(work), 256, 0, stream>>>(g, (const T*)x, (T*)y, argmax)
  DT_SWITCH(dtype, F);
#undef F
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_maxpool2d_cl_bwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* dy,
                                      const unsigned char* argmax, void* dx, hipStream_t stream) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g) || !argmax) return -1;
  const long work = (long)N * H * W * (C / 8);
#define F(T) maxpool_cl_bwd<T><<<grid_for(work), 256, 0, stream>>>(g, (const T*)dy, argmax, (T*)dx)
  DT_SWITCH(dtype, F);
#undef F
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_dwconv2d_cl_fwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x,
                                     const float* w, void* z, hipStream_t stream) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g) || !w) return -1;
  const long work = (long)N * g.Ho * g.Wo * (C / 8);
  const bool buf = dw_buf_ok((long)N * H * W * C, dtype == CMHAR_F32 ? 4 : 2);
#define FK(T, KK)                                                                                               \
  do {                                                                                                          \
    if (buf) dwconv_cl_fwd<T, KK, true><<<grid_for(work), 256, 0, stream>>>(g, (const T*)x, w, (T*)z);          \
    else dwconv_cl_fwd<T, KK, false><<<grid_for(work), 256, 0, stream>>>(g, (const T*)x, w, (T*)z);             \
  } while (0)
#define F(T) do { if (k == 3) FK(T, 3); else if (k == 2) FK(T, 2); else FK(T, 1); } while (0)
  DT_SWITCH(dtype, F);
#undef F
#undef FK
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_dwconv2d_cl_dgrad(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* dz,
                                       const float* w, void* dx, hipStream_t stream) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g) || !w) return -1;
  const long work = (long)N * H * W * (C / 8);
  const bool buf = dw_buf_ok((long)N * g.Ho * g.Wo * C, dtype == CMHAR_F32 ? 4 : 2);
#define FK(T, KK)                                                                                               \
  do {                                                                                                          \
    if (buf) dwconv_cl_dgrad<T, KK, true><<<grid_for(work), 256, 0, stream>>>(g, (const T*)dz, w, (T*)dx);      \
    else dwconv_cl_dgrad<T, KK, false><<<grid_for(work), 256, 0, stream>>>(g, (const T*)dz, w, (T*)dx);         \
  } while (0)
#define F(T) do { if (k == 3) FK(T, 3); else if (k == 2) FK(T, 2); else FK(T, 1); } while (0)
  DT_SWITCH(dtype, F);
#undef F
#undef FK
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" long cmhar_dwconv2d_cl_wgrad_ws(int N, int H, int W, int C, int k, int s, int p) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g)) return -1;
  return (long)dw_chunks((long)N * g.Ho * g.Wo) * k * k * C;
}

extern "C" int cmhar_dwconv2d_cl_wgrad(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x,
                                       const void* dz, float* dw, float* ws, hipStream_t stream) {
  const Pool g = make_pool(N, H, W, C, k, s, p);
  if (!pool_ok(g) || !dw || !ws || C > 2048) return -1;
  const long M = (long)N * g.Ho * g.Wo;
  const int nch = dw_chunks(M);
  const int rpc = (int)((M + nch - 1) / nch);
  const bool buf = dw_buf_ok((long)N * H * W * C, dtype == CMHAR_F32 ? 4 : 2);
#define FK(T, KK)                                                                                               \
  do {                                                                                                          \
    if (buf) dwconv_cl_wgrad_partial<T, KK, true><<<nch, 256, 0, stream>>>(g, rpc, (const T*)x, (const T*)dz, ws); \
    else dwconv_cl_wgrad_partial<T, KK, false><<<nch, 256, 0, stream>>>(g, rpc, (const T*)x, (const T*)dz, ws);    \
  } while (0)
#define F(T) do { if (k == 3) FK(T, 3); else if (k == 2) FK(T, 2); else FK(T, 1); } while (0)
  DT_SWITCH(dtype, F);
#undef F
#undef FK
  dwconv_cl_wgrad_final<<<dim3(cdiv(C, 32), k * k), 256, 0, stream>>>(C, k * k, nch, ws, dw);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// One pack's plan: channel tile ci_t, 8-channel vector form, grid; false on invalid arguments
static bool pack_plan(int Cout, int Cin, int kt, int kh, int kw, int Kp, const float* w, const void* out,
                      const void* out_flip, int& taps, int& ci_t, bool& v8, dim3& grid) {
  if (Cout <= 0 || Cin <= 0 || kt <= 0 || kh <= 0 || kw <= 0 || !w || (!out && !out_flip)) return false;
  taps = kt * kh * kw;
  if (out && Kp < taps * Cin) return false;
  if (PACK_CO * taps > PACK_LDS) return false;
  ci_t = max(1, min(Cin, min(32, PACK_LDS / (PACK_CO * taps))));
  v8 = Cin % 8 == 0 && Cout % 8 == 0 && (!out || Kp % 8 == 0) && ci_t >= 8;
  if (v8) ci_t &= ~7;
  grid = dim3(cdiv(Cout, PACK_CO), cdiv(Cin, ci_t));
  return true;
}

extern "C" int cmhar_conv_pack_weights(int out_dtype, int n, const int* dims, const void* const* ptrs,
                                       hipStream_t stream) {
  if (n < 0 || (n > 0 && (!dims || !ptrs))) return -1;
  if (out_dtype != CMHAR_BF16 && out_dtype != CMHAR_F32) return -1;
  for (int i0 = 0; i0 < n; i0 += PACK_JOBS) {
    PackJobs jobs{};
    jobs.n = min(PACK_JOBS, n - i0);
    int blocks = 0;
    for (int k = 0; k < jobs.n; ++k) {
      const int* d = dims + 6 * (i0 + k);
      const void* const* pp = ptrs + 3 * (i0 + k);
      int taps, ci_t;
      bool v8;
      dim3 g;
      if (!pack_plan(d[0], d[1], d[2], d[3], d[4], d[5], (const float*)pp[0], pp[1], pp[2], taps, ci_t, v8, g))
        return -1;
      jobs.j[k] = PackJob{(const float*)pp[0], const_cast<void*>(pp[1]), const_cast<void*>(pp[2]), d[0], d[1], taps,
                          d[5], ci_t, (int)g.x, blocks, (int)v8, pack_div(taps)};
      blocks += (int)(g.x * g.y);
    }
    if (out_dtype == CMHAR_BF16) conv_pack_multi_kernel<bf16><<<blocks, 256, 0, stream>>>(jobs);
    else conv_pack_multi_kernel<float><<<blocks, 256, 0, stream>>>(jobs);
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_conv_pack_weight(int out_dtype, int Cout, int Cin, int kt, int kh, int kw, int Kp, const float* w,
                                      void* out, void* out_flip, hipStream_t stream) {
  int taps, ci_t;
  bool v8;
  dim3 grid;
  if (!pack_plan(Cout, Cin, kt, kh, kw, Kp, w, out, out_flip, taps, ci_t, v8, grid)) return -1;
#define F(T)                                                                                                       \
  if (v8)                                                                                                          \
    conv_pack_kernel<T, true><<<grid, 256, 0, stream>>>(Cout, Cin, taps, Kp, ci_t, pack_div(taps), w, (T*)out,     \
                                                        (T*)out_flip);                                             \
  else                                                                                                             \
    conv_pack_kernel<T, false><<<grid, 256, 0, stream>>>(Cout, Cin, taps, Kp, ci_t, pack_div(taps), w, (T*)out,    \
                                                         (T*)out_flip)
  DT_SWITCH(out_dtype, F);
#undef F
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_conv_grad_unpack(int Cout, int Cin, int R, int kw, int Kp, int rs, int cs, const float* src,
                                      float* dst, hipStream_t stream) {
  if (Cout <= 0 || Cin <= 0 || R <= 0 || kw <= 0 || rs <= 0 || cs <= 0 || !src || !dst) return -1;
  if ((long)(R - 1) * rs + (long)(kw - 1) * cs + Cin > Kp) return -1;
  const long n = (long)Cout * Cin * R * kw;
  const long dmax = max(kw, max(R, Cin));
  if (n * dmax >= (1L << 32)) return -2;       // PackDiv exactness bound
  conv_grad_unpack_kernel<<<grid_for(n), 256, 0, stream>>>((unsigned)n, Cin, R, kw, Kp, rs, cs, pack_div(kw),
                                                           pack_div(R), pack_div(Cin), src, dst);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
