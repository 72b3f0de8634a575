// Shared device helpers for the cmhar HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(8))) short short8_t;
typedef __attribute__((ext_vector_type(4))) float floatx4;
typedef __attribute__((ext_vector_type(16))) float floatx16;
typedef __attribute__((ext_vector_type(4))) unsigned uint4_t;
typedef __attribute__((ext_vector_type(2))) unsigned uint2_t;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// dtype codes used across the C ABI
enum { CMHAR_F32 = 0, CMHAR_BF16 = 1, CMHAR_F16 = 2 };

// activation / epilogue codes
enum {
  ACT_NONE = 0,
  ACT_GELU = 1,        // out = gelu_erf(acc + bias); aux_out (optional) = acc + bias
  ACT_RELU = 2,        // out = relu(acc + bias)
  ACT_DGELU = 3,       // out = acc * gelu_erf'(aux_in)
  ACT_DRELU = 4,       // out = acc * (aux_in > 0)
  ACT_GELU_SAVEGRAD = 5,  // out = gelu_erf(acc + bias); aux_out = gelu_erf'(acc + bias)
  ACT_MULAUX = 6,      // out = acc * aux_in   (the GELU backward against a saved derivative)
};

// The epilogue struct is part of the C ABI (include/cmhar.h); every extern "C" definition in csrc/ is checked
// against its declaration there because each translation unit includes the header.
#include "cmhar.h"
typedef CmharEpilogue Epilogue;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

template <typename T> __device__ __forceinline__ float to_f(T x);
template <> __device__ __forceinline__ float to_f<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f<bf16>(bf16 x) { return (float)x; }
template <> __device__ __forceinline__ float to_f<f16>(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }

// 16-bit MFMA operands travel as raw 16-B fragments (bf16x8 carriers: LDS-DMA, ds_read and the transposing
// ds_read_tr16 move bits, not numbers); E picks the number format the matrix core reads them in — bf16 for training,
// fp16 for the fp16 inference path (BASELINE config 5).
template <typename E> __device__ __forceinline__ floatx4 mma16(bf16x8 a, bf16x8 b, floatx4 c);
template <> __device__ __forceinline__ floatx4 mma16<bf16>(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <> __device__ __forceinline__ floatx4 mma16<f16>(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
template <typename E> __device__ __forceinline__ floatx16 mma32(bf16x8 a, bf16x8 b, floatx16 c);
template <> __device__ __forceinline__ floatx16 mma32<bf16>(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <> __device__ __forceinline__ floatx16 mma32<f16>(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// 8 fp32 values → one 16-B fragment in format E
template <typename E> __device__ __forceinline__ bf16x8 pack_frag8(const float (&x)[8]) {
  typedef E __attribute__((ext_vector_type(8))) v8;
  v8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (E)x[j];
  return __builtin_bit_cast(bf16x8, v);
}

// GELU(erf) and its derivative from ONE shared set of transcendentals.  Φ(x) = ½·erfc(−x/√2) with erfc(z), z ≥ 0,
// from the Chebyshev-fitted form erfc(z) = t·exp(−z² + R(t)), t = 1/(1 + z/2) (Numerical Recipes `erfcc`,
// relative error < 1.2e-7 for every z, so the x < 0 tail keeps full relative precision — no 1 − erf cancellation).
// exp(−z²) = exp(−x²/2) is also the Gaussian density factor of Φ'(x), so gelu and gelu' cost 2 v_exp + 1 v_rcp
// + ~14 FMA-class ops together (ocml erff alone is a branchy ~25-op polynomial).
__device__ __forceinline__ void gelu_pair(float x, float& g, float& gp) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float r = 0.17087277f;
  r = fmaf(r, t, -0.82215223f);
  r = fmaf(r, t, 1.48851587f);
  r = fmaf(r, t, -1.13520398f);
  r = fmaf(r, t, 0.27886807f);
  r = fmaf(r, t, -0.18628806f);
  r = fmaf(r, t, 0.09678418f);
  r = fmaf(r, t, 0.37409196f);
  r = fmaf(r, t, 1.00002368f);
  r = fmaf(r, t, -1.26551223f);
  const float e1 = __expf(-0.5f * x * x);          // exp(−z²)
  const float half_erfc = 0.5f * t * e1 * __expf(r);  // Φ(−|x|)
  const float cdf = x < 0.f ? half_erfc : 1.0f - half_erfc;
  g = x * cdf;
  gp = fmaf(x, 0.39894228040143268f * e1, cdf);
}
__device__ __forceinline__ float gelu_erf(float x) { float g, gp; gelu_pair(x, g, gp); return g; }
__device__ __forceinline__ float gelu_erf_grad(float x) { float g, gp; gelu_pair(x, g, gp); return gp; }

// The same pair for 16-bit outputs: erfc(z) ≈ t·P4(t)·exp(−z²), t = 1 / (1 + 0.3275911 z) (Abramowitz–Stegun 7.1.26)
// — one transcendental and four FMAs fewer than the Chebyshev form above; its absolute error in Φ and Φ′·x + Φ
// (≤ 4.3e-7 / 3.2e-7 over [−12, 12], the Chebyshev form's 3.8e-7 / 2.9e-7) is ~10⁴× below a bf16 ulp of values
// ≥ 1e-3, so the stored GELU / GELU′ are the same numbers to bf16 resolution.  The FC1 forward epilogue (GELU and
// GELU′ of 154 M elements per launch) is VALU-bound with every CU in it at once.
__device__ __forceinline__ void gelu_pair16(float x, float& g, float& gp) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = 1.061405429f;
  p = fmaf(p, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e1 = __expf(-0.5f * x * x);          // exp(−z²)
  const float half_erfc = 0.5f * t * p * e1;       // Φ(−|x|)
  const float cdf = x < 0.f ? half_erfc : 1.0f - half_erfc;
  g = x * cdf;
  gp = fmaf(x, 0.39894228040143268f * e1, cdf);
}
// gelu_pair16 on two values at once, written in packed-fp32 form (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 do two
// lanes' worth per instruction; the reciprocal, exp2 and the sign select stay per value): the FC1 forward epilogue
// evaluates it 154 M times per launch with the matrix pipes idle.  Same approximation as gelu_pair16 with its ½ folded
// into P and exp(−x²/2) as exp2(x²·(−½·log2 e)) — results within its error bound (tests/test_kernels_gpu.py GELU
// tests), not bit-identical to it.
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ void gelu_pair16x2(f32x2 x, f32x2& g, f32x2& gp) {
  // ed = φ(x) = exp(−x²/2)/√(2π) from one exp2 (the 1/√(2π) as a log2 offset), so Φ(−|x|) = t·P(t)·exp(−x²/2) =
  // t·(P(t)·√(2π)/2)·ed — P's coefficients carry ½·√(2π) — and GELU′ = x·φ(x) + Φ(x) is one fma
  constexpr float kS = 0.5f * 2.5066282746310002f;    // ½·√(2π)
  const f32x2 t = {__builtin_amdgcn_rcpf(fmaf(fabsf(x[0]), 0.70710678118654752f * 0.3275911f, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(x[1]), 0.70710678118654752f * 0.3275911f, 1.0f))};
  f32x2 p = {kS * 1.061405429f, kS * 1.061405429f};
  p = __builtin_elementwise_fma(p, t, f32x2{kS * -1.453152027f, kS * -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2{kS * 1.421413741f, kS * 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2{kS * -0.284496736f, kS * -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2{kS * 0.254829592f, kS * 0.254829592f});
  // log2(φ(x)) = x²·(−½·log2 e) + log2(1/√(2π))
  const f32x2 arg = __builtin_elementwise_fma(x * x, f32x2{-0.5f * 1.4426950408889634f, -0.5f * 1.4426950408889634f},
                                              f32x2{-1.3257480647361593f, -1.3257480647361593f});
  const f32x2 ed = {__builtin_amdgcn_exp2f(arg[0]), __builtin_amdgcn_exp2f(arg[1])};   // φ(x)
  const f32x2 h = t * p * ed;                                                         // Φ(−|x|)
  const f32x2 om = f32x2{1.0f, 1.0f} - h;
  const f32x2 cdf = {x[0] < 0.f ? h[0] : om[0], x[1] < 0.f ? h[1] : om[1]};
  g = x * cdf;
  gp = __builtin_elementwise_fma(x, ed, cdf);
}

template <typename OutT>
__device__ __forceinline__ void gelu_pair_for(float x, float& g, float& gp) {
  if constexpr (sizeof(OutT) == 2) gelu_pair16(x, g, gp);
  else gelu_pair(x, g, gp);
}
template <typename OutT> __device__ __forceinline__ float gelu_for(float x) { float g, gp; gelu_pair_for<OutT>(x, g, gp); return g; }
template <typename OutT> __device__ __forceinline__ float gelu_grad_for(float x) { float g, gp; gelu_pair_for<OutT>(x, g, gp); return gp; }

// Counter-hash dropout mask shared by every kernel that applies or regenerates an element dropout:
// keep (m, n) iff hash(seed, m, n) / 2^32 >= p; kept values are scaled by 1/(1-p) (nn.Dropout semantics).
__device__ __forceinline__ unsigned drop_hash(unsigned long long seed, unsigned long long a, unsigned b) {
  unsigned long long x = seed ^ (0x9E3779B97F4A7C15ull * (a + 1)) ^ (0xC2B2AE3D27D4EB4Full * (b + 1));
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (unsigned)x;
}
__device__ __forceinline__ float drop_mask(unsigned long long seed, float p, long row, int col) {
  if (p <= 0.f) return 1.f;
  const float u = (float)drop_hash(seed, (unsigned long long)row, (unsigned)col) * 2.3283064365386963e-10f;
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// Apply the epilogue to one accumulator element at (m, n).  OutT = float or bf16.
template <typename OutT>
__device__ __forceinline__ void epilogue_store(const Epilogue& e, OutT* __restrict__ C, long ldc, int m, int n,
                                               float acc) {
  float v = e.alpha * acc;
  if (e.bias) v += e.bias[n];
  if (e.rowadd) v += e.rowadd[(long)(m % e.rowadd_mod) * e.rowadd_ld + n];
  if (n >= e.colscale_lo && n < e.colscale_hi) v *= e.colscale;
  switch (e.act) {
    case ACT_GELU:
      if (e.aux_out) ((OutT*)e.aux_out)[(long)m * e.ldo + n] = from_f<OutT>(v);
      v = gelu_for<OutT>(v);
      break;
    case ACT_RELU: v = v > 0.f ? v : 0.f; break;
    case ACT_DGELU: v *= gelu_grad_for<OutT>(to_f<OutT>(((const OutT*)e.aux_in)[(long)m * e.lda + n])); break;
    case ACT_DRELU: v = to_f<OutT>(((const OutT*)e.aux_in)[(long)m * e.lda + n]) > 0.f ? v : 0.f; break;
    case ACT_GELU_SAVEGRAD: {
      float g, gp;
      gelu_pair_for<OutT>(v, g, gp);
      if (e.aux_out) ((OutT*)e.aux_out)[(long)m * e.ldo + n] = from_f<OutT>(gp);
      v = g;
      break;
    }
    case ACT_MULAUX: v *= to_f<OutT>(((const OutT*)e.aux_in)[(long)m * e.lda + n]); break;
    default: break;
  }
  if (e.pdrop > 0.f) v *= drop_mask(e.seed, e.pdrop, m, n);
  if (e.residual) v += to_f<OutT>(((const OutT*)e.residual)[(long)m * e.ldr + n]);
  OutT* p = C + (long)m * ldc + n;
  if (e.beta != 0.f) v += e.beta * to_f<OutT>(*p);
  *p = from_f<OutT>(v);
}

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

// XCD-aware bijective block remap: workgroups are dispatched round-robin over the 8 XCDs by linear block id, so
// id → (id % 8)'s contiguous chunk of the logical index space; logically adjacent blocks (sharing operand panels,
// or the K/V of one attention head) then run on one XCD and share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// (block, head, batch) of a flash-attention workgroup on a (blocks, H, B) grid, with every block of one (batch, head)
// on the same XCD (K/V, or Q/dO, of that head is then fetched into one L2 and re-read from it by the head's other
// blocks).
struct BlkIdx { int blk, hd, b; };
__device__ __forceinline__ BlkIdx flash_block(int H) {
  const int nb = gridDim.x;
  const int lin = blockIdx.x + nb * (blockIdx.y + gridDim.y * blockIdx.z);
  const int r = xcd_remap(lin, nb * gridDim.y * gridDim.z);
  const int bh = r / nb;
  return {r % nb, bh % H, bh / H};
}

// The exact-fp32 parity mode runs its large GEMMs and its D = 64 attention on the f32-input MFMA; CMHAR_F32_MFMA=0
// (read once per process) routes them to the exact-f32 VALU kernels instead (A/B tests: identical GEMM bits).
static inline bool cmhar_f32_mfma() {
  static const bool on = [] {
    const char* v = getenv("CMHAR_F32_MFMA");
    return !(v && v[0] == '0');
  }();
  return on;
}

#define CMHAR_CHECK_LAUNCH() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
