// bf16 MFMA GEMM for gfx950 with fused epilogues — the VideoMAE Linear / tubelet-conv hot path.
//
// C[m,n] = epilogue( sum_k A(m,k) * B(k,n) ), bf16 operands, fp32 accumulation in MFMA accumulators.
// Operand layouts are template parameters so that ONE kernel body covers the three GEMMs of a Linear:
//   forward  Y  = X  · Wᵀ : A = X  [M][K] (K-contiguous), B = W  [N][K] (K-contiguous)
//   dgrad    dX = dY · W  : A = dY [M][N] (K-contiguous), B = W  [N][K] (N-contiguous: contraction on rows)
//   wgrad    dW = dYᵀ· X  : A = dY [M][N] (M-contiguous), B = X  [M][K] (K-contiguous ... along rows)
// K-contiguous tiles are read with ds_read_b128; row-contraction tiles with the gfx950 transposing
// ds_read_b64_tr_b16, so no operand is ever transposed in HBM.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2, 64x64 per wave = 4x4 mfma_f32_16x16x32_bf16), LDS double buffer
// (2 x 32 KiB), register-staged global->LDS copy with XOR-swizzled images (bank-conflict-free for both read
// kinds), one barrier per K-tile, XCD-aware block remap.  Split-K writes fp32 partial slabs that
// cmhar_splitk_reduce combines with the epilogue.
#include "common.h"

#include <map>
#include <mutex>
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

// K-contiguous image: [128 rows][64 k] = 8 chunks of 16 B per row; chunk ^= (row>>1)&7.
__device__ __forceinline__ int kc_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// Row-contraction image: [64 k][128 cols] = 16 chunks per row; chunk ^= 2*((k&3) | ((k>>3)&1)<<2).
__device__ __forceinline__ int mc_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int mc_off(int k, int chunk) { return k * 256 + ((chunk ^ mc_swz(k)) << 4); }

template <bool KC>
struct Stage {
  uint4_t r[4];
  unsigned ok = 0xfu;   // in-range bits of r (BOUNDS loads)
  // Load this operand's tile (rows r0.., k0..) into registers; rows = M or N index.  BOUNDS: rows / k past the
  // matrix edge read a clamped (valid) address — never a branch around a load — and are zeroed when the tile is
  // written to LDS: a select on the value right after the load makes the compiler wait for that load there, before
  // the compute the register prefetch is meant to overlap (conv3d.hip, kLateZero).
  template <bool BOUNDS>
  __device__ __forceinline__ void load(const bf16* __restrict__ P, long ld, int rows_total, int r0, int k0,
                                       int kend, int tid) {
    if (BOUNDS) ok = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int c = it * NT + tid;
      int row, kk;
      if (KC) { row = c >> 3; kk = (c & 7) * 8; } else { kk = c >> 4; row = (c & 15) * 8; }
      const int gr = r0 + row, gk = k0 + kk;
      if (BOUNDS) {
        const bool in = gr < rows_total && gk < kend;
        const bf16* src = in ? (KC ? (P + (long)gr * ld + gk) : (P + (long)gk * ld + gr)) : P;
        r[it] = *(const uint4_t*)src;
        ok |= (unsigned)in << it;
      } else {
        r[it] = *(const uint4_t*)(KC ? (P + (long)gr * ld + gk) : (P + (long)gk * ld + gr));
      }
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int c = it * NT + tid;
      int off;
      if (KC) off = kc_off(c >> 3, c & 7); else off = mc_off(c >> 4, c & 15);
      *(uint4_t*)(lds + off) = (ok >> it) & 1 ? r[it] : uint4_t{0u, 0u, 0u, 0u};
    }
  }
};

// Fragment of 16 rows (r0 + lane&15) x 32 k (kk*32 + 8*(lane>>4) + j) for the 16x16x32 MFMA.
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* lds, int r0, int kk, int lane) {
  if (KC) {
    const int row = r0 + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    return *(const bf16x8*)(lds + kc_off(row, chunk));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (r0 >> 3) + (p >> 1);
    short4_t lo, hi;
    {
      const int k = kk * 32 + 8 * g + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + mc_off(k, chunk) + (p & 1) * 8));
    }
    {
      const int k = kk * 32 + 8 * g + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + mc_off(k, chunk) + (p & 1) * 8));
    }
    short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}


// 8 consecutive elements of an OutT row as fp32 / back, with single 16-B (bf16) or 2 x 16-B (fp32) accesses.
// The epilogue's streamed 16-bit operands (aux_in, residual: each element read once) and the split-K reduce's slabs
// are loaded non-temporal, like the outputs are stored: step 696.8 / 696.5 -> 700.1 / 701.4 clips/s with both
// (tools/debug/lib_step_ab.sh, alternated on one box; each alone half of that).  CMHAR_NT_EPI_LOAD /
// CMHAR_NT_REDUCE_LOAD = 0: plain loads.
#ifndef CMHAR_NT_EPI_LOAD
#define CMHAR_NT_EPI_LOAD 1
#endif
template <typename OutT>
__device__ __forceinline__ void load8(const OutT* __restrict__ p, float (&x)[8], bool nt = false) {
  if constexpr (sizeof(OutT) == 2) {
    typedef OutT __attribute__((ext_vector_type(8))) v8;
    typedef int __attribute__((ext_vector_type(4))) i4;
    const v8 v = (CMHAR_NT_EPI_LOAD && nt) ? __builtin_bit_cast(v8, __builtin_nontemporal_load((const i4*)p))
                                           : *(const v8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (float)v[j];
  } else {
    const floatx4 a = *(const floatx4*)p, b = *(const floatx4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { x[j] = a[j]; x[4 + j] = b[j]; }
  }
}
// 16-bit epilogue outputs (C and aux_out) are stored non-temporal: written once, read by a later kernel, they no
// longer displace this GEMM's operand panels from L2.  Measured in the bench step (tools/debug/lib_step_ab.sh,
// alternated on one box): 684.2 / 685.4 -> 700.0 / 701.6 clips/s (QKV forward 206 -> 192 us, FC1 forward 363 -> 338);
// bit-identical outputs.  The same for the 8-phase kernel's fp32 split-K slabs (re-read by the reduce) was slower
// (693 clips/s), and for the bf16 Vec8 stores of the norm / elementwise kernels neutral.  CMHAR_NT_STORE=0: plain.
#ifndef CMHAR_NT_STORE
#define CMHAR_NT_STORE 1
#endif
template <typename OutT>
__device__ __forceinline__ void store8(OutT* __restrict__ p, const float (&x)[8]) {
  if constexpr (sizeof(OutT) == 2) {
    typedef OutT __attribute__((ext_vector_type(8))) v8;
    v8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (OutT)x[j];
    if (CMHAR_NT_STORE) {
      typedef int __attribute__((ext_vector_type(4))) i4;
      __builtin_nontemporal_store(__builtin_bit_cast(i4, v), (i4*)p);
    } else {
      *(v8*)p = v;
    }
  } else {
    *(floatx4*)p = floatx4{x[0], x[1], x[2], x[3]};
    *(floatx4*)(p + 4) = floatx4{x[4], x[5], x[6], x[7]};
  }
}

// Vectorised epilogue for 8 consecutive columns n0..n0+7 of row m: every operand is moved with 16-B accesses
// (callers guarantee 16-B alignment: N % 8 == 0 on this path, leading dimensions % 8 == 0, checked on the host).
// Each optional stage is a wave-uniform branch on a kernel argument.
// The [M,N] 16-bit operand an epilogue streams per element — aux_in of act 3 / 4 / 6, else the residual — or null.
// Kernels instantiated with PFS (launched only for epilogues that have one) load it two row groups ahead of its use,
// the first two under the accumulator staging, and hand each row's vector to epilogue_store8 as `pre`.
#ifndef CMHAR_EPI_PF2
#define CMHAR_EPI_PF2 1
#endif
// row groups loaded ahead (2, 4, 6 or 8; A/B knob)
#ifndef CMHAR_EPI_PFD
#define CMHAR_EPI_PFD 8
#endif
// CMHAR_EPI_BIAS_HOIST (8-phase kernel): the bias loaded once per epilogue pass, not per row (the C stores may
// alias e.bias as far as the compiler knows, so it reloads it for every row: QKV forward 192.5 -> 183.3 us)
#ifndef CMHAR_EPI_BIAS_HOIST
#define CMHAR_EPI_BIAS_HOIST 1
#endif
// CMHAR_EPI_XPASS (depth 8 only): the second pass's operand loaded during the first pass (FC2 dgrad 311 -> 303 us)
#ifndef CMHAR_EPI_XPASS
#define CMHAR_EPI_XPASS 1
#endif
template <typename OutT>
__device__ __forceinline__ const OutT* epi_stream(const Epilogue& e, long& ld) {
  if (e.act == ACT_DGELU || e.act == ACT_DRELU || e.act == ACT_MULAUX) { ld = e.lda; return (const OutT*)e.aux_in; }
  ld = e.ldr;
  return (const OutT*)e.residual;
}
static inline bool epi_has_stream(const Epilogue& e) {
  return e.residual != nullptr || e.act == ACT_DGELU || e.act == ACT_DRELU || e.act == ACT_MULAUX;
}
// an epilogue that reads any per-element or per-row operand (the persistent kernel's exclusion, persist_ok)
static inline bool epi_reads(const Epilogue& e) { return epi_has_stream(e) || e.rowadd != nullptr || e.beta != 0.f; }
template <typename OutT>
__device__ __forceinline__ void decode8(const uint4_t& r, float (&x)[8]) {
  typedef OutT __attribute__((ext_vector_type(8))) v8;
  const v8 v = __builtin_bit_cast(v8, r);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)v[j];
}

template <typename OutT>
__device__ __forceinline__ void epilogue_store8(const Epilogue& e, OutT* __restrict__ C, long ldc, int m, int n0,
                                                float (&v)[8], bool has_pre = false,
                                                uint4_t pre = uint4_t{0u, 0u, 0u, 0u}, const floatx4* bpre = nullptr) {
  // bpre: this thread's 8 bias values, loaded once per pass by the caller (the kernel's own C stores may alias
  // e.bias as far as the compiler knows, so it would reload them for every row, a dependent L2 round trip)
  // pre (has_pre): this row's 8 values of epi_stream(e), already loaded (16-bit OutT only)
  const bool pre_aux = has_pre && (e.act == ACT_DGELU || e.act == ACT_DRELU || e.act == ACT_MULAUX);
  float x[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = e.alpha * v[j];
  if (e.bias) {
    const floatx4 b0 = bpre ? bpre[0] : *(const floatx4*)(e.bias + n0);
    const floatx4 b1 = bpre ? bpre[1] : *(const floatx4*)(e.bias + n0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { x[j] += b0[j]; x[4 + j] += b1[j]; }
  }
  if (e.rowadd) {
    const float* r = e.rowadd + (long)(m % e.rowadd_mod) * e.rowadd_ld + n0;
    const floatx4 r0 = *(const floatx4*)r, r1 = *(const floatx4*)(r + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { x[j] += r0[j]; x[4 + j] += r1[j]; }
  }
  if (n0 >= e.colscale_lo && n0 < e.colscale_hi) {    // the range is a multiple of 8 columns (host-checked)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] *= e.colscale;
  }
  if (e.act == ACT_GELU) {
    if (e.aux_out) store8<OutT>((OutT*)e.aux_out + (long)m * e.ldo + n0, x);
    if constexpr (sizeof(OutT) == 2) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2 g, gp;
        gelu_pair16x2(f32x2{x[j], x[j + 1]}, g, gp);
        x[j] = g[0];
        x[j + 1] = g[1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = gelu_for<OutT>(x[j]);
    }
  } else if (e.act == ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fmaxf(x[j], 0.f);
  } else if (e.act == ACT_DGELU) {
    if constexpr (sizeof(OutT) == 2) {
      if (pre_aux) decode8<OutT>(pre, t); else load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    } else {
      load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    }
    if constexpr (sizeof(OutT) == 2) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2 g, gp;
        gelu_pair16x2(f32x2{t[j], t[j + 1]}, g, gp);
        x[j] *= gp[0];
        x[j + 1] *= gp[1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] *= gelu_grad_for<OutT>(t[j]);
    }
  } else if (e.act == ACT_DRELU) {
    if constexpr (sizeof(OutT) == 2) {
      if (pre_aux) decode8<OutT>(pre, t); else load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    } else {
      load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = t[j] > 0.f ? x[j] : 0.f;
  } else if (e.act == ACT_GELU_SAVEGRAD) {
    if constexpr (sizeof(OutT) == 2) {   // the FC1 forward: packed-fp32 form (gelu_pair16x2)
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2 g, gp;
        gelu_pair16x2(f32x2{x[j], x[j + 1]}, g, gp);
        x[j] = g[0];
        x[j + 1] = g[1];
        t[j] = gp[0];
        t[j + 1] = gp[1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gelu_pair_for<OutT>(x[j], x[j], t[j]);
    }
    if (e.aux_out) store8<OutT>((OutT*)e.aux_out + (long)m * e.ldo + n0, t);
  } else if (e.act == ACT_MULAUX) {
    if constexpr (sizeof(OutT) == 2) {
      if (pre_aux) decode8<OutT>(pre, t); else load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    } else {
      load8<OutT>((const OutT*)e.aux_in + (long)m * e.lda + n0, t, true);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] *= t[j];
  }
  if (e.pdrop > 0.f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] *= drop_mask(e.seed, e.pdrop, m, n0 + j);
  }
  if (e.residual) {
    if constexpr (sizeof(OutT) == 2) {
      if (has_pre && !pre_aux) decode8<OutT>(pre, t);
      else load8<OutT>((const OutT*)e.residual + (long)m * e.ldr + n0, t, true);
    } else {
      load8<OutT>((const OutT*)e.residual + (long)m * e.ldr + n0, t, true);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += t[j];
  }
  OutT* dst = C + (long)m * ldc + n0;
  if (e.beta != 0.f) {
    load8<OutT>(dst, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += e.beta * t[j];
  }
  store8<OutT>(dst, x);
}

// ---------------------------------------------------------------------------------------------------------------
// Register-direct epilogue of the 256² kernels (CMHAR_EPI_DIRECT = 1; instantiations without a streamed epilogue
// operand).  The K loop runs with the MFMA operands swapped — acc = (B fragment) x (A fragment), i.e. Cᵀ per 16x16
// block, the same products in the same order (bit-identical) — so lane l holds in acc[i][j][r] ONE row
// (i*16 + (l&15)) and FOUR consecutive columns (j*16 + 4*(l>>4) + r) of the wave's 128x64 block.  A v_permlane16_swap
// per accumulator register pairs blocks (2p, 2p+1) and a row_ror:8 DPP exchange pairs the lane halves (pair_rows), so
// every store instruction covers 8 rows x 128 contiguous bytes straight from registers — no LDS staging round trip
// (64 4-B ds_writes per lane per pass, a wait, the read-back).  fp32 partial slabs (raw) need no pairing: a block's 4
// columns are one 16-B store.  Measured in the bench step (rocprofv3 per launch, tools/debug/trace_ab.sh): FC2 forward
// (tail split) -3 %, weight gradients -1 to -2.5 %, the plain forward epilogues within +-1.5 %; the epilogues that
// stream a 16-bit operand (residual, GELU') were 11-20 % SLOWER with every prefetch depth tried (4, 8, all 16 segments
// before the first store) — the legacy loop's LDS staging is what hides those loads — so the PFS instantiations keep
// the staged epilogue.
// ablation builds of the persistent kernel (tools/debug): 1 = K-tile 2's DMA wait leaves the previous tile's stores in
// flight (racy: timing only), 2 = no epilogue
#ifndef CMHAR_PERSIST_ABL
#define CMHAR_PERSIST_ABL 0
#endif
// CMHAR_PERSIST_PROBE (debug builds, tools/debug/persist_probe.py): in-kernel s_memtime stamps of wave 0 / wave 4 of
// every workgroup around each tile boundary, read back by cmhar_debug_persist_probe
#ifndef CMHAR_PERSIST_PROBE
#define CMHAR_PERSIST_PROBE 0
#endif
#if CMHAR_PERSIST_PROBE
__device__ unsigned long long g_persist_probe[256 * 12 * 2 * 6];
#endif
// start-time stagger of the persistent kernel's workgroups, in units of s_sleep(127) (~8 k cycles) per quarter
#ifndef CMHAR_PERSIST_STAGGER
#define CMHAR_PERSIST_STAGGER 0
#endif
#ifndef CMHAR_EPI_DIRECT
#define CMHAR_EPI_DIRECT 1
#endif
// segments of the streamed operand in flight (even, 2..8): all 128 accumulators stay live across the rolled epilogue
// loop
#ifndef CMHAR_EPI_DIRECT_PD
#define CMHAR_EPI_DIRECT_PD 8
#endif
// acc += (x-fragment) · (w-fragment) in the accumulator layout the epilogue expects
template <typename E, bool DIRECT>
__device__ __forceinline__ floatx4 mma_ab(bf16x8 a, bf16x8 b, floatx4 c) {
  return DIRECT ? mma16<E>(b, a, c) : mma16<E>(a, b, c);
}
// Row block i of the accumulators (16 rows x the wave's 64 columns) as two store segments of 8 whole rows each.
// After the permlane16 pairing a lane holds row li = l&15, 8 columns at 32p + cofs(g) for p = 0 (v0) and 1 (v1); a
// row_ror:8 DPP exchange between the lane halves li < 8 / li >= 8 then gives segment X = rows 0-7 (lanes li < 8 keep
// their p = 0 columns, lanes li >= 8 take the p = 1 columns of row li - 8) and segment Y = rows 8-15 (the mirror), so
// that every store instruction covers 8 rows x 128 contiguous bytes, the legacy staging loop's pattern (16 rows x 64 B
// per instruction measured 3-4 % slower in the step: 730 -> 710 clips/s).  Lane l of a segment: row (l & 7) (+8 for Y),
// columns 32*((l >> 3) & 1) + cofs(l >> 4) .. +7.  A switch on the (wave-uniform) block index with a static accumulator
// access in every case keeps the epilogue loop rolled — fully unrolled, the inlined epilogue_store8 bodies took the
// kernels from ~4.5 k to 14-18 k instructions (past the instruction cache), and a dynamic acc index put acc in scratch.
__device__ __forceinline__ float dpp_ror8(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));   // row_ror:8
}
__device__ __forceinline__ void pair_rows(const floatx4 (&acc)[8][4], int i, bool lo, float (&x)[8], float (&y)[8]) {
  float v0[8], v1[8];
  auto take = [&](const floatx4(&a)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const auto s0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[0][r]), __float_as_uint(a[1][r]), false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[2][r]), __float_as_uint(a[3][r]), false, false);
      v0[r] = __uint_as_float(s0[0]);
      v0[4 + r] = __uint_as_float(s0[1]);
      v1[r] = __uint_as_float(s1[0]);
      v1[4 + r] = __uint_as_float(s1[1]);
    }
  };
  switch (i) {
    case 0: take(acc[0]); break;
    case 1: take(acc[1]); break;
    case 2: take(acc[2]); break;
    case 3: take(acc[3]); break;
    case 4: take(acc[4]); break;
    case 5: take(acc[5]); break;
    case 6: take(acc[6]); break;
    default: take(acc[7]); break;
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const float got = dpp_ror8(lo ? v1[r] : v0[r]);   // lanes li < 8 send v1 and receive v0 of row li + 8
    x[r] = lo ? v0[r] : got;
    y[r] = lo ? got : v1[r];
  }
}
// m0 / n0: the wave block's first row / column; raw (fp32 partials of the wave block's first row, row stride raw_ld)
// or null for the product epilogue.  PFS: the epilogue's streamed 16-bit operand (epi_stream) is loaded PD segments
// ahead of its use (the first PD before the first store).
// The epilogues epi_direct's fast path takes: alpha 1, no dropout, nothing read (residual, aux_in, rowadd, beta),
// no activation or the GELU pair with its GELU' output (16-bit outputs only)
__host__ __device__ inline bool epi_fast_ok(const Epilogue& e) {
  return e.alpha == 1.f && e.pdrop <= 0.f && !e.residual && !e.aux_in && !e.rowadd && e.beta == 0.f &&
         (e.act == ACT_NONE || (e.act == ACT_GELU_SAVEGRAD && e.aux_out));
}
// The epilogues the persistent kernel takes (epi_persist): alpha 1, no dropout / rowadd / beta; either nothing else,
// the GELU pair with its GELU' output, the product with a 16-bit aux_in (ACT_MULAUX: FC2's input gradient × GELU'), or
// a 16-bit residual
__host__ __device__ inline bool epi_persist_ok(const Epilogue& e) {
  if (e.alpha != 1.f || e.pdrop > 0.f || e.rowadd || e.beta != 0.f) return false;
  if (e.act == ACT_NONE) return !e.aux_in;
  if (e.act == ACT_GELU_SAVEGRAD) return e.aux_out && !e.residual && !e.aux_in;
  if (e.act == ACT_MULAUX) return e.aux_in && !e.residual;
  return false;
}
// This lane's 8 bias columns (zeros without a bias): an unconditional load (a dummy valid address without one), so
// that no load is left pending on a path the compiler cannot rule out — a loop-carried pending load of a persistent
// kernel's epilogue made hipcc wait vmcnt before the next tile's first MFMAs (WAW on the load's registers).
__device__ __forceinline__ void epi_bias(const Epilogue& e, const void* dummy, int n0, int lane, floatx4 (&bh)[2]) {
  const int g = lane >> 4, li = lane & 15;
  const int cn = n0 + 32 * (li >> 3) + (((g & 1) << 4) | ((g >> 1) << 3));
  const float* p = e.bias ? e.bias + cn : (const float*)dummy;
  bh[0] = *(const floatx4*)p;
  bh[1] = *(const floatx4*)(p + 4);
}
// FAST_ONLY: the caller guarantees the fast path's epilogue (epi_fast_ok) — the generic per-element path is not
// compiled in (the persistent kernel: its registers are at the limit)
template <typename OutT, bool PFS, bool BIAS_IN = false, bool FAST_ONLY = false>
__device__ __forceinline__ void epi_direct(const Epilogue& e, OutT* __restrict__ C, long ldc, float* __restrict__ raw,
                                           long raw_ld, int m0, int n0, int lane, const floatx4 (&acc)[8][4],
                                           const floatx4* bias_in = nullptr) {
  const int g = lane >> 4, li = lane & 15;
  if (raw) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) *(floatx4*)(raw + (long)(i * 16 + li) * raw_ld + j * 16 + 4 * g) = acc[i][j];
    return;
  }
  const bool lo = li < 8;
  const int cn = n0 + 32 * (li >> 3) + (((g & 1) << 4) | ((g >> 1) << 3));   // this lane's 8 columns, both segments
  const int rl = m0 + (li & 7);                                              // this lane's row in segment X of block 0
  floatx4 bh[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  if constexpr (BIAS_IN) {   // loaded by epi_bias and already zeroed without a bias by the caller
    bh[0] = bias_in[0];
    bh[1] = bias_in[1];
  } else if (e.bias) {
    bh[0] = *(const floatx4*)(e.bias + cn);
    bh[1] = *(const floatx4*)(e.bias + cn + 4);
  }
  // Fast path (16-bit output; bias, key-column scale, GELU pair — the persistent kernel's launches): packed-fp32
  // math on the two segments and nothing else per element.  The in-kernel timeline (tools/debug/persist_probe.py)
  // showed the generic epilogue VALU-bound: 12.6-15.7 k cycles per QKV tile (~26 % of the tile) for 16 stores per
  // wave — a wave64 VALU instruction holds its SIMD 4 cycles, and epilogue_store8's per-element alpha multiply,
  // bias add, colscale select and row / column address arithmetic ran ~150 instructions per 16 values.
  if constexpr (sizeof(OutT) == 2 && !PFS) {
    const bool gp = e.act == ACT_GELU_SAVEGRAD && e.aux_out;
    if (FAST_ONLY || epi_fast_ok(e)) {
      typedef __attribute__((ext_vector_type(2))) float f2;
      f2 b2[4], s2 = {1.f, 1.f};
#pragma unroll
      for (int k = 0; k < 4; ++k) b2[k] = f2{bh[k >> 1][2 * (k & 1)], bh[k >> 1][2 * (k & 1) + 1]};
      const bool cs = cn >= e.colscale_lo && cn < e.colscale_hi;   // a multiple-of-8 range: whole segments
      if (cs) s2 = f2{e.colscale, e.colscale};
      const bool any_cs = e.colscale_hi > e.colscale_lo;
      OutT* const c0 = C + (long)rl * ldc + cn;
      OutT* const a0 = gp ? (OutT*)e.aux_out + (long)rl * e.ldo + cn : nullptr;
      auto seg = [&](const float (&v)[8], OutT* dst, OutT* adst) __attribute__((always_inline)) {
        f2 x[4], t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          x[k] = f2{v[2 * k], v[2 * k + 1]} + b2[k];
          if (any_cs) x[k] = x[k] * s2;
          if (gp) gelu_pair16x2(x[k], x[k], t[k]);
        }
        typedef OutT __attribute__((ext_vector_type(2))) o2;
        typedef int __attribute__((ext_vector_type(4))) i4;
        i4 o, a;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = __builtin_bit_cast(int, __builtin_convertvector(x[k], o2));
          if (gp) a[k] = __builtin_bit_cast(int, __builtin_convertvector(t[k], o2));
        }
        if (CMHAR_NT_STORE) {
          if (gp) __builtin_nontemporal_store(a, (i4*)adst);
          __builtin_nontemporal_store(o, (i4*)dst);
        } else {
          if (gp) *(i4*)adst = a;
          *(i4*)dst = o;
        }
      };
#pragma unroll 1
      for (int i = 0; i < 8; ++i) {
        float x[8], y[8];
        pair_rows(acc, i, lo, x, y);
        const long ro = (long)i * 16 * ldc, ra = gp ? (long)i * 16 * e.ldo : 0;
        seg(x, c0 + ro, a0 + ra);
        seg(y, c0 + ro + 8 * ldc, a0 + ra + 8 * e.ldo);
      }
      return;
    }
  }
  if constexpr (FAST_ONLY) return;
  long pld = 0;
  const OutT* const ps = PFS && sizeof(OutT) == 2 ? epi_stream<OutT>(e, pld) : nullptr;
  // segment c = 2i + h: row rl + 16i + 8h
  auto pf = [&](int c) -> uint4_t {
    return ps ? *(const uint4_t*)(ps + (long)(rl + c * 8) * pld + cn) : uint4_t{0u, 0u, 0u, 0u};
  };
  constexpr int PD = CMHAR_EPI_DIRECT_PD;
  uint4_t pw[PD];
#pragma unroll
  for (int j = 0; j < PD; ++j) pw[j] = PFS ? pf(j) : uint4_t{0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    const uint4_t q0 = pw[0], q1 = pw[1];
    if constexpr (PFS) {
#pragma unroll
      for (int j = 0; j + 2 < PD; ++j) pw[j] = pw[j + 2];
      if (2 * i + PD < 16) {
        pw[PD - 2] = pf(2 * i + PD);
        pw[PD - 1] = pf(2 * i + PD + 1);
      }
    }
    float x[8], y[8];
    pair_rows(acc, i, lo, x, y);
    // the column index made opaque per iteration: hoisted out of the loop, the column-dependent parts of the
    // epilogue (the dropout hash's per-column terms, 64-bit column offsets) sat in 32+ VGPRs next to the 128 live
    // accumulators and spilled
    int nc = cn;
    asm volatile("" : "+v"(nc));
    const int m = rl + i * 16;
    epilogue_store8<OutT>(e, C, ldc, m, nc, x, ps != nullptr, q0, bh);
    epilogue_store8<OutT>(e, C, ldc, m + 8, nc, y, ps != nullptr, q1, bh);
  }
}

constexpr int EPI_LD = BN + 4;                       // padded fp32 staging row: conflict-free acc writes
constexpr int SMEM_BYTES = BM * EPI_LD * 4;          // 67584 B ≥ the 64 KiB of double-buffered A/B stages

template <typename E, bool A_KC, bool B_KC, typename OutT, bool BOUNDS>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(int M, int N, int K, const bf16* __restrict__ A, long lda,
                                                          const bf16* __restrict__ B, long ldb,
                                                          OutT* __restrict__ C, long ldc, Epilogue e, int klen,
                                                          long split_stride, int raw_out, int row0 = 0) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  // stage buffers: A at smem + 16K*buf, B at smem + 32K + 16K*buf
#define As(buf) (smem + 16384 * (buf))
#define Bs(buf) (smem + 32768 + 16384 * (buf))
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // row0: this launch covers output rows row0 .. M-1 only (the tail rows after a 256² launch over the full rounds)
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M - row0 + BM - 1) / BM;
  // split index folded into the XCD remap: one XCD runs whole splits, whose CUs then share each K-slice in L2
  const int ntile = tiles_m * tiles_n;
  const int rlin = xcd_remap(blockIdx.x + ntile * blockIdx.z, ntile * gridDim.z);
  const int bid = rlin % ntile, split = rlin / ntile;
  // row-major tile order: the blocks an XCD runs together share A row panels while the whole (small) weight
  // matrix stays resident in that XCD's L2 — activations are streamed from HBM once
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int bm = row0 + tm * BM, bn = tn * BN;
  const int kbeg = split * klen;
  const int kend = min(K, kbeg + klen);
  C += (long)split * split_stride;

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  Stage<A_KC> sa;
  Stage<B_KC> sb;
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    sa.template load<BOUNDS>(A, lda, M, bm, kbeg, kend, tid);
    sb.template load<BOUNDS>(B, ldb, N, bn, kbeg, kend, tid);
    sa.store(As(0), tid);
    sb.store(Bs(0), tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.template load<BOUNDS>(A, lda, M, bm, kbeg + (kt + 1) * BK, kend, tid);
      sb.template load<BOUNDS>(B, ldb, N, bn, kbeg + (kt + 1) * BK, kend, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<A_KC>(As(cur), wr * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<B_KC>(Bs(cur), wc * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16<E>(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      sa.store(As(cur ^ 1), tid);
      sb.store(Bs(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // Epilogue: stage the fp32 tile through LDS (static accumulator indexing — the accumulators stay in
  // registers through the main loop), then every thread emits 8 consecutive columns per row with 16-B stores.
  float* T = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wr * 64 + i * 16 + 4 * (lane >> 4) + r) * EPI_LD + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int cg = (tid & 15) * 8;        // 16 threads x 8 columns per row
  const int n0 = bn + cg;
  for (int rr = tid >> 4; rr < BM; rr += NT / 16) {
    const int m = bm + rr;
    if (m >= M) break;
    float v[8];
    const floatx4 lo = *(const floatx4*)&T[rr * EPI_LD + cg], hi = *(const floatx4*)&T[rr * EPI_LD + cg + 4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
    if (raw_out) {
      float* dst = (float*)C + (long)m * ldc + n0;
      if (!BOUNDS || n0 + 8 <= N) {
        *(floatx4*)dst = lo;
        *(floatx4*)(dst + 4) = hi;
      } else {
        for (int j = 0; j < 8 && n0 + j < N; ++j) dst[j] = v[j];
      }
    } else if (!BOUNDS || n0 + 8 <= N) {
      epilogue_store8<OutT>(e, C, ldc, m, n0, v);
    } else {
      for (int j = 0; j < 8 && n0 + j < N; ++j) epilogue_store<OutT>(e, C, ldc, m, n0 + j, v[j]);
    }
  }
}

#undef As
#undef Bs

// the split-K reduce reads its slabs non-temporal (see CMHAR_NT_EPI_LOAD)
#ifndef CMHAR_NT_REDUCE_LOAD
#define CMHAR_NT_REDUCE_LOAD 1
#endif
// slabs whose loads the reduce keeps in flight together (A/B knob; 8 measured the same as 4 on the weight-gradient
// reduces in round 6: QKV / FC1 / FC2 wgrad + reduce 176.4 / 226.4 / 239.2 vs 177.0 / 227.0 / 237.5 us)
#ifndef CMHAR_REDUCE_DEPTH
#define CMHAR_REDUCE_DEPTH 4
#endif
// Sum split-K fp32 partial slabs and apply the epilogue; 8 consecutive columns per thread when N % 8 == 0.
// m_base: the slabs hold rows m_base .. m_base+M-1 of C (tail-split hybrid); 0 for a plain split-K GEMM.
template <typename OutT>
__global__ void splitk_reduce_kernel(int M, int N, int splits, const float* __restrict__ P, long split_stride,
                                     OutT* __restrict__ C, long ldc, Epilogue e, int m_base = 0) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((N & 7) == 0) {
    const long e0 = idx * 8;
    if (e0 >= (long)M * N) return;
    const int m = (int)(e0 / N) + m_base, n0 = (int)(e0 % N);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto ld = [&](int z, floatx4& a, floatx4& b) {
      if (CMHAR_NT_REDUCE_LOAD) {   // the slabs are dead after this pass
        a = __builtin_nontemporal_load((const floatx4*)(P + z * split_stride + e0));
        b = __builtin_nontemporal_load((const floatx4*)(P + z * split_stride + e0 + 4));
      } else {
        a = *(const floatx4*)(P + z * split_stride + e0);
        b = *(const floatx4*)(P + z * split_stride + e0 + 4);
      }
    };
    auto add = [&](const floatx4& a, const floatx4& b) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { s[j] += a[j]; s[4 + j] += b[j]; }
    };
    // RD slabs' loads in flight before they are added in slab order (one pair per iteration left the reduce
    // latency-bound); same order of additions, same bits
    constexpr int RD = CMHAR_REDUCE_DEPTH;
    int z = 0;
    for (; z + RD - 1 < splits; z += RD) {
      floatx4 a[RD], b[RD];
#pragma unroll
      for (int u = 0; u < RD; ++u) ld(z + u, a[u], b[u]);
#pragma unroll
      for (int u = 0; u < RD; ++u) add(a[u], b[u]);
    }
    for (; z < splits; ++z) {
      floatx4 a, b;
      ld(z, a, b);
      add(a, b);
    }
    if (e.rowsum && idx < M) {                       // bias-gradient slabs follow the C slabs
      float r = 0.f;
      for (int z = 0; z < splits; ++z) r += P[splits * split_stride + (long)z * M + idx];
      e.rowsum[idx] = e.rowsum_beta != 0.f ? r + e.rowsum_beta * e.rowsum[idx] : r;
    }
    epilogue_store8<OutT>(e, C, ldc, m, n0, s);
    return;
  }
  const long total = (long)M * N;
  if (idx >= total) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += P[z * split_stride + idx];
  epilogue_store<OutT>(e, C, ldc, m, n, s);
}

static inline int reduce_blocks(int M, int N) {
  const long total = (long)M * N;
  return (N & 7) == 0 ? cdiv(cdiv(total, 8), 256) : cdiv(total, 256);
}

// ---------------------------------------------------------------------------------------------------------------
// 256x256x64 tile, 512 threads = 8 waves (2 x 4, 128x64 outputs per wave = 8x4 mfma_f32_16x16x32_bf16 blocks),
// operands staged by LDS-DMA (global_load_lds_dwordx4: 16 B per lane straight into LDS, no VGPR round trip, no
// ds_write), two 64 KiB LDS buffers: tile k+1 streams in while tile k is consumed; one barrier per K-tile.
// The XOR swizzles are applied on the per-lane GLOBAL source address (the DMA's LDS destination is lane-linear)
// and the same swizzles on the fragment reads.  Used when M, N % 256 == 0 and K (per split) % 64 == 0 — every
// VideoMAE-B GEMM at 16×224² and 16×112².
// ---------------------------------------------------------------------------------------------------------------
constexpr int TM2 = 256, TN2 = 256, TK2 = 64, NT2 = 512;
constexpr int EPI2_LD = 68;                                  // per-wave 64x64 fp32 staging row (+4 pad)
constexpr int SMEM2 = 8 * 64 * EPI2_LD * 4;                  // 139264 B ≥ 2 x 64 KiB operand buffers

__device__ __forceinline__ int mc_off512(int k, int chunk) { return k * 512 + ((chunk ^ mc_swz(k)) << 4); }

typedef __attribute__((address_space(3))) void* lds_void_ptr;

#ifndef CMHAR_GEMM8P_ASM_DMA
#define CMHAR_GEMM8P_ASM_DMA 1
#endif
// One 1-KiB LDS-DMA piece (`buffer_load_dwordx4 … lds`, 16 B per lane) issued by inline asm: hipcc then does not see
// an LDS write in flight, so it no longer puts `s_waitcnt vmcnt(0)` in front of every transposed LDS read
// (ds_read_b64_tr_b16) that follows a DMA issue — in the 8-phase weight-gradient instantiation it did so at every
// phase, draining the next K-tile's prefetch three times per K-tile (asm issue: weight gradients 14–19 % faster,
// `gpurun_out/r04w_gemm_ab.log`).  Used by the instantiations with transposed reads (CMHAR_GEMM8P_ASM_DMA = 0: the
// builtin everywhere).  The kernel orders every DMA itself (counted vmcnt +
// barriers, as with the builtin).  src: the tile origin at this K-slice (wave-uniform).  M0 is written here without
// the compiler knowing (M0 is a reserved register: clang accepts it on a clobber list only with a warning that the
// clobber may not be honoured), so an instantiation that issues its DMA this way must contain NO compiler-generated
// M0 use: both operands of a kernel take the same kAD choice, and the one builtin LDS-DMA that could share a K loop
// with it (gemm256's L2 prefetch, CMHAR_GEMM_L2PF) is compiled out of kAD instantiations (static_assert there).
__device__ __forceinline__ void dma_asm(const char* src, char* lds, int voff) {
  const unsigned long long a = (unsigned long long)src;
  uint4_t rs;
  rs[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  rs[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) & 0xffffu;
  rs[2] = 0x7fffffffu;
  rs[3] = 0x00020000u;
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void_ptr)lds);
  // (s_nop: the SALU write of M0 needs one wait state before the LDS-DMA reads it — hipcc puts the same nop after
  // its own M0 writes; inside inline asm its hazard recognizer cannot)
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" :: "s"(la), "v"(voff), "s"(rs)
               : "memory");
}


// LDS-DMA source of one operand (256 rows/cols x 64 k per tile) as a BUFFER load: the scalar resource holds the
// tile's K-slice origin (advanced per K-tile with two SALU ops), the per-lane byte offsets of this wave's 4 pieces
// (swizzle included) are computed once, so issuing a piece costs no VALU at all (`buffer_load_dwordx4 … lds`).
// (The `global_load_lds` form needs a 64-bit per-lane address per piece: 2 `v_lshl_add_u64` + a move each, 8 pieces
// per wave per K-tile.)
template <bool KC>
struct DmaSrc {
  const char* base;   // operand + tile origin (bytes)
  long kstride;       // bytes per k step
  int voff[4];
  int pf_off;         // L2 prefetch: this lane's 128-B line of a tile (see l2_prefetch)
  __device__ __forceinline__ void init(const bf16* __restrict__ P, long ld, int r0, int wave, int lane) {
    {   // tile line idx (0..255) = this thread's index within its operand's half of the workgroup
      const int idx = (wave & 3) * 64 + lane;
      pf_off = KC ? (int)((long)idx * ld * 2) : (int)((long)(idx >> 2) * ld * 2 + (idx & 3) * 128);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int i = wave * 4 + t;                          // 1 KiB piece index (32 per tile)
      if (KC) {   // [256 rows][64 k]: piece = 8 rows of 128 B
        const int row = 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        voff[t] = (int)(((long)row * ld + lc * 8) * 2);
      } else {    // [64 k][256 cols]: piece = 2 k-rows of 512 B
        const int k = 2 * i + (lane >> 5);
        const int lc = (lane & 31) ^ mc_swz(k);
        voff[t] = (int)(((long)k * ld + lc * 8) * 2);
      }
    }
    base = (const char*)(KC ? P + (long)r0 * ld : P + r0);
    kstride = KC ? 2 : ld * 2;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(int k0) const {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)k0 * kstride), (short)0, 0x7fffffff, 0x00020000);
  }
  // Issue one of this wave's 4 pieces (t = 0..3).
  __device__ __forceinline__ void piece(__amdgpu_buffer_rsrc_t r, char* lds, int wave, int t) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(lds + (wave * 4 + t) * 1024), 16, voff[t], 0, 0, 0);
  }
  template <bool ASM = false>
  __device__ __forceinline__ void tile(int k0, char* lds, int wave) const {
    if constexpr (ASM) {
#pragma unroll
      for (int t = 0; t < 4; ++t) dma_asm(base + (long)k0 * kstride, lds + (wave * 4 + t) * 1024, voff[t]);
    } else {
      const __amdgpu_buffer_rsrc_t r = rsrc(k0);
#pragma unroll
      for (int t = 0; t < 4; ++t) piece(r, lds, wave, t);
    }
  }
  // Touch every 128-B line of the tile at k0 (256 lines, one per lane of 4 waves) with a 4-byte LDS-DMA into a junk
  // LDS slot: the lines are pulled into this XCD's L2 a tile ahead of the DMA that stages them, so that DMA hits L2.
  __device__ __forceinline__ void l2_prefetch(int k0, char* junk) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(k0), (lds_void_ptr)junk, 4, pf_off, 0, 0, 0);
  }
};

// L2 prefetch of K-tile kt+2 in the two-buffer weight-gradient K loop (CMHAR_GEMM_L2PF=1; A/B knob, off: measured
// 12 % SLOWER on the VideoMAE weight gradients — 242.6 vs 216.6 µs average in the step trace — the extra line
// requests cost more L2 / TA issue than the misses they pre-empt)
#ifndef CMHAR_GEMM_L2PF
#define CMHAR_GEMM_L2PF 0
#endif

template <bool KC>
__device__ __forceinline__ bf16x8 frag256(const char* lds, int r0, int kk, int lane) {
  if (KC) {
    const int row = r0 + (lane & 15);
    return *(const bf16x8*)(lds + kc_off(row, kk * 4 + (lane >> 4)));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (r0 >> 3) + (p >> 1);
    const int k = kk * 32 + 8 * g + q;
    const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + mc_off512(k, chunk) + (p & 1) * 8));
    const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + mc_off512(k + 4, chunk) + (p & 1) * 8));
    short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// MODE (ablation builds only, tools/debug): 0 = product; 3 = epilogue only (no K loop); 4 = K loop only (no
// epilogue); 5 = LDS staging only; 6 = staging + plain bf16 stores; 7 = K loop without the LDS-DMA (stale
// operands), no epilogue; 8 = as 4 (the spread-DMA ablation it named is recorded in DESIGN.md).
// NA: A-operand LDS buffers.  2 = tile k+1 streams in while tile k is consumed (A and B double-buffered, 128 KiB);
// 3 = the A tile (the HBM-streamed activation panel) is fetched TWO tiles ahead — three 32 KiB A buffers + two
// 32 KiB B buffers = the whole 160 KiB LDS — so its longer HBM/MALL latency has two K-tiles of MFMAs to hide under.
template <typename E, bool A_KC, bool B_KC, typename OutT, int MODE = 0, int NA = 2, bool PFS = false>
__global__ __launch_bounds__(NT2, 2) void gemm256_kernel(int M, int N, int K, const bf16* __restrict__ A, long lda,
                                                         const bf16* __restrict__ B, long ldb, OutT* __restrict__ C,
                                                         long ldc, Epilogue e, int klen, long split_stride,
                                                         int raw_out, float* __restrict__ sk_ws, int n_dp,
                                                         int sk_klen) {
  constexpr bool kAD = CMHAR_GEMM8P_ASM_DMA && (!A_KC || !B_KC);   // see dma_asm
  constexpr bool kDirect = CMHAR_EPI_DIRECT && MODE == 0 && !PFS;   // register-direct epilogue (epi_direct)
  // the L2 prefetch is a builtin LDS-DMA (compiler-managed M0): never in a K loop whose DMA the asm issues
  constexpr bool PF = CMHAR_GEMM_L2PF && NA == 2 && MODE == 0 && !kAD;
  static_assert(!(PF && kAD), "builtin LDS-DMA (L2 prefetch) beside asm-issued DMA: M0 is not tracked across dma_asm");
  __shared__ __attribute__((aligned(16))) char smem[NA == 3 ? 163840 : SMEM2 + (PF ? 2048 : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = N / TN2, tiles_m = M / TM2;
  const int ntile = tiles_m * tiles_n;
  int bid, split, kbeg, kend;
  bool sk = false;
  if (n_dp > 0) {
    // Tail split (data-parallel + split-K hybrid): blocks [0, n_dp) are whole tiles (full rounds of the chip); the
    // remaining tail tiles — whole tile rows, n_dp is row-aligned — are split along K over the rest of the grid so
    // the last round fills the CUs; their fp32 partials go to sk_ws and splitk_reduce applies the epilogue.
    if ((int)blockIdx.x < n_dp) {
      bid = xcd_remap(blockIdx.x, n_dp);
      split = 0;
      kbeg = 0;
      kend = K;
    } else {
      const int n_tail = ntile - n_dp;
      const int u = xcd_remap(blockIdx.x - n_dp, gridDim.x - n_dp);
      bid = n_dp + u % n_tail;
      split = u / n_tail;
      kbeg = split * sk_klen;
      kend = min(K, kbeg + sk_klen);
      sk = true;
    }
  } else {
    // split index folded into the XCD remap: one XCD runs whole splits, whose CUs then share each K-slice in L2
    const int rlin = xcd_remap(blockIdx.x + ntile * blockIdx.z, ntile * gridDim.z);
    bid = rlin % ntile;
    split = rlin / ntile;
    kbeg = split * klen;
    kend = min(K, kbeg + klen);
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int bm = tm * TM2, bn = tn * TN2;
  const int tail_m0 = (n_dp / max(tiles_n, 1)) * TM2;
  const long sk_stride = (long)(M - tail_m0) * N;
  float* const rs_slab = raw_out ? (float*)C + (long)gridDim.z * split_stride + (long)split * M : nullptr;
  C += (long)split * split_stride;
  const int nk = MODE >= 3 && MODE != 4 && MODE != 7 && MODE != 8 ? 0 : (kend - kbeg) / TK2;
  // Weight-gradient GEMMs (A = dYᵀ, M-contiguous) can also emit the bias gradient Σ_k A(m,k): one extra MFMA of an
  // A fragment against an all-ones B fragment.  One block per row panel (tn == tm % tiles_n, spreading the panels
  // over the column tiles) does it, each of its waves for 2 of its 8 A fragments: +2 MFMAs per 32 on those blocks.
  const bool rs = !A_KC && e.rowsum != nullptr && tn == tm % tiles_n;
  const float one8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const bf16x8 ones = pack_frag8<E>(one8);
  floatx4 accb[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Software-pipelined K loop.  Per K-tile of 64 (two 32-deep MFMA steps kk = 0, 1):
  //   issue the LDS-DMA of tile kt+1 into the other buffer;
  //   kk = 0: 32 MFMAs, each A slot refilled with its kk = 1 fragment once its 4 MFMAs have issued;
  //   kk = 1, A rows 0-3: 16 MFMAs;
  //   sync point: vmcnt(0) (own DMA of kt+1 landed) + lgkmcnt(0) (own reads of tile kt done) + barrier;
  //     then tile kt+1's kk = 0 fragments are read into the freed slots WHILE
  //   kk = 1, A rows 4-7: the last 16 MFMAs of tile kt still run.
  // So the post-barrier LDS read latency hides under MFMAs instead of stalling all 8 waves at every barrier.
  bf16x8 af[8], bf0[4], bf1[4];
  auto load_k0 = [&](const char* a_s, const char* b_s, int i_lo, int i_hi, bool with_b) {
    if (with_b) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bf0[j] = frag256<B_KC>(b_s, wc * 64 + j * 16, 0, lane);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i >= i_lo && i < i_hi) af[i] = frag256<A_KC>(a_s, wr * 128 + i * 16, 0, lane);
  };
  auto a_buf = [&](int t) -> char* { return NA == 3 ? smem + (t % 3) * 32768 : smem + (t & 1) * 65536; };
  auto b_buf = [&](int t) -> char* { return NA == 3 ? smem + 98304 + (t & 1) * 32768 : smem + (t & 1) * 65536 + 32768; };
  DmaSrc<A_KC> da;
  DmaSrc<B_KC> db;
  da.init(A, lda, bm, wave, lane);
  db.init(B, ldb, bn, wave, lane);
  if (nk > 0) {
    if (MODE != 7) {
      da.template tile<kAD>(kbeg, a_buf(0), wave);
      db.template tile<kAD>(kbeg, b_buf(0), wave);
      if (NA == 3 && nk > 1) da.template tile<kAD>(kbeg + TK2, a_buf(1), wave);
    }
    // tile 0 landed (own pieces) before the barrier — explicitly: with the asm-issued DMA (kAD) hipcc no longer adds
    // the vmcnt(0) it used to put in front of the first transposed read
    if (NA == 3 && nk > 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    load_k0(a_buf(0), b_buf(0), 0, 8, true);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf1[j] = frag256<B_KC>(b_buf(0), wc * 64 + j * 16, 1, lane);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const char* a_s = a_buf(kt);
    const bool more = kt + 1 < nk;
    const bool more2 = NA == 3 && kt + 2 < nk;
    char* nxt = a_buf(kt + 1);
    char* nxt_b = b_buf(kt + 1);
    // B(kt+1) first, A(kt+2) second (NA = 3): vmcnt counts in issue order, so waiting for B(kt+1) (and the A(kt+1)
    // issued a tile earlier) can leave A(kt+2)'s 4 pieces in flight.  (Spreading the 8 pieces one per 4-MFMA group
    // instead of this burst measured neutral on forward/dgrad and 1.3-1.7x slower on the NA = 2 weight-gradient layout,
    // whose vmcnt(0) then waits on the last, late piece.)
    const bool pf = PF && kt + 2 < nk;
    if (MODE != 7) {
      if (NA == 3) {
        if (more) db.template tile<kAD>(kbeg + (kt + 1) * TK2, nxt_b, wave);
        if (more2) da.template tile<kAD>(kbeg + (kt + 2) * TK2, a_buf(kt + 2), wave);
      } else if (more) {
        da.template tile<kAD>(kbeg + (kt + 1) * TK2, nxt, wave);
        db.template tile<kAD>(kbeg + (kt + 1) * TK2, nxt_b, wave);
        if (pf) {       // after the DMA pieces: the vmcnt(1) below leaves this one in flight
          if (wave < 4) da.l2_prefetch(kbeg + (kt + 2) * TK2, smem + SMEM2 + wave * 256);
          else db.l2_prefetch(kbeg + (kt + 2) * TK2, smem + SMEM2 + wave * 256);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mma_ab<E, kDirect>(af[i], bf0[j], acc[i][j]);
      if (!A_KC && rs && wc == (i >> 1))
        accb[i & 1] = mma16<E>(af[i], ones, accb[i & 1]);
      af[i] = frag256<A_KC>(a_s, wr * 128 + i * 16, 1, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mma_ab<E, kDirect>(af[i], bf1[j], acc[i][j]);
      if (!A_KC && rs && wc == (i >> 1))
        accb[i & 1] = mma16<E>(af[i], ones, accb[i & 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      // own DMA of tile kt+1 landed, own reads of tile kt returned; then everyone's
      if (more2) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (pf) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      load_k0(nxt, nxt_b, 0, 4, true);                     // slots 0-3 and bf0 are free now
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 4; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mma_ab<E, kDirect>(af[i], bf1[j], acc[i][j]);
      if (!A_KC && rs && wc == (i >> 1))
        accb[i & 1] = mma16<E>(af[i], ones, accb[i & 1]);
      if (more) af[i] = frag256<A_KC>(nxt, wr * 128 + i * 16, 0, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bf1[j] = frag256<B_KC>(nxt_b, wc * 64 + j * 16, 1, lane);
    }
  }
  if (!A_KC && rs && (lane & 15) == 0) {       // every column of a ones-product holds the row sum: lanes 0,16,32,48
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wr * 128 + (2 * wc + ii) * 16 + 4 * (lane >> 4) + r;
        if (rs_slab) rs_slab[m] = accb[ii][r];
        else e.rowsum[m] = e.rowsum_beta != 0.f ? accb[ii][r] + e.rowsum_beta * e.rowsum[m] : accb[ii][r];
      }
  }
  if constexpr (kDirect) {
    float* raw = raw_out ? (float*)C + (long)(bm + wr * 128) * ldc + bn + wc * 64
                 : sk ? sk_ws + split * sk_stride + (long)(bm + wr * 128 - tail_m0) * N + bn + wc * 64 : nullptr;
    epi_direct<OutT, PFS>(e, C, ldc, raw, raw_out ? ldc : N, bm + wr * 128, bn + wc * 64, lane, acc);
    return;
  }
  __syncthreads();
  if (MODE == 4 || MODE == 7 || MODE == 8) {   // keep every accumulator live, store nothing
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) ((float*)C)[tid] = t;
    return;
  }

  // epilogue: per wave, two passes of 64x64 through a private LDS slab, 16-B stores
  float* T = (float*)(smem + wave * 64 * EPI2_LD * 4);
  long pld = 0;
  const OutT* const ps = PFS && sizeof(OutT) == 2 && !raw_out && !sk ? epi_stream<OutT>(e, pld) : nullptr;
  // XP: the second pass's operand is loaded during the first pass (after its staging), not at its own start
  constexpr bool XP = PFS && CMHAR_EPI_PFD == 8 && CMHAR_EPI_XPASS;
  uint4_t pwn[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pwn[j] = uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int cg = (lane & 7) * 8;
    const int n0 = bn + wc * 64 + cg;
    auto pf = [&](int it) -> uint4_t {
      return ps ? *(const uint4_t*)(ps + (long)(bm + wr * 128 + pass * 64 + it * 8 + (lane >> 3)) * pld + n0)
                : uint4_t{0u, 0u, 0u, 0u};
    };
    constexpr int PD = CMHAR_EPI_PFD;   // row groups in flight (even, 2..8)
    uint4_t pw[PD];                      // pw[j]: the operand of row group it2 + j (static indices only)
#pragma unroll
    for (int j = 0; j < PD; ++j) pw[j] = PFS && !(XP && pass == 1) ? pf(j) : pwn[j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(i * 16 + 4 * (lane >> 4) + r) * EPI2_LD + j * 16 + (lane & 15)] = acc[pass * 4 + i][j][r];
    // the slab is private to this wave and a wave's LDS operations complete in order: no workgroup barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (XP && pass == 0 && ps) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pwn[j] = *(const uint4_t*)(ps + (long)(bm + wr * 128 + 64 + j * 8 + (lane >> 3)) * pld + n0);
    }
    auto row = [&](int it, uint4_t pre) __attribute__((always_inline)) {
      const int rr = it * 8 + (lane >> 3);
      const int m = bm + wr * 128 + pass * 64 + rr;
      const floatx4 lo = *(const floatx4*)&T[rr * EPI2_LD + cg], hi = *(const floatx4*)&T[rr * EPI2_LD + cg + 4];
      if (MODE == 5) {
        if (lo[0] + hi[3] == 1234.5f) ((float*)C)[tid] = lo[1];
      } else if (MODE == 6) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) { o[j] = (bf16)lo[j]; o[4 + j] = (bf16)hi[j]; }
        *(bf16x8*)((bf16*)C + (long)m * ldc + n0) = o;
      } else if (raw_out) {
        float* dst = (float*)C + (long)m * ldc + n0;
        *(floatx4*)dst = lo;
        *(floatx4*)(dst + 4) = hi;
      } else if (sk) {
        float* dst = sk_ws + split * sk_stride + (long)(m - tail_m0) * N + n0;
        *(floatx4*)dst = lo;
        *(floatx4*)(dst + 4) = hi;
      } else {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
        epilogue_store8<OutT>(e, C, ldc, m, n0, v, ps != nullptr, pre);
      }
    };
    if constexpr (PFS) {
#pragma unroll 1
      for (int it2 = 0; it2 < 8; it2 += 2) {
        const uint4_t q0 = pw[0], q1 = pw[1];
#pragma unroll
        for (int j = 0; j + 2 < PD; ++j) pw[j] = pw[j + 2];
        if (it2 + PD < 8) {
          pw[PD - 2] = pf(it2 + PD);
          pw[PD - 1] = pf(it2 + PD + 1);
        }
        row(it2, q0);
        row(it2 + 1, q1);
      }
    } else {
#pragma unroll 2
      for (int it = 0; it < 8; ++it) row(it, pw[0]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this pass' slab reads done before the next overwrite
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Forward and dgrad layouts (A K-contiguous), whole K: the same 256² tile and wave layout, but the K loop is an
// 8-interval-per-K-tile ping-pong.  The two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7 — one of each on
// every SIMD) run one barrier interval apart, so in every interval one wave of each SIMD issues its 16 MFMAs (one
// 64x32 quadrant of its 128x64 block, K = 64, at s_setprio 1) while the other issues its LDS fragment reads and
// LDS-DMA pieces.  Per K-tile a wave runs 4 phases = quadrants (0,0) (0,1) (1,1) (1,0), reading A0+B0, B1, A1,
// nothing.  Staging: K-tile t+1's A lower half is DMA'd in phase 1 of t, both B halves in phase 2; after phase 4's
// vmcnt(0) (everything of t+1 landed) the A upper half of t+2 is issued into the buffer t just finished with (its
// last read was group 0's phase 3, two intervals earlier).  Every region is restaged >= 2 intervals after its last
// read and read >= 1 interval after the wait that retires it.  (Measured against gemm256_kernel in one process,
// tools/debug/gemm_ab.py: forward 5-6 % faster at K = 768-1536; bit-identical — each output's k order is unchanged.)
// ---------------------------------------------------------------------------------------------------------------
// Per-lane offsets of this wave's 2 pieces of each half of an operand tile.  K-contiguous [256 rows][64 k]: half h =
// rows 128h..128h+127.  Row-contraction [64 k][256 cols] (the dgrad weight operand): half h = k rows 32h..32h+31.
template <bool KC>
struct DmaHalf {
  const char* base;
  long kstride;
  int voff[2][2];
  __device__ __forceinline__ void init(const bf16* __restrict__ P, long ld, int r0, int wave, int lane) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int i = 16 * h + 2 * wave + t;                   // 1 KiB piece index within the tile image
        if (KC) {
          const int row = 8 * i + (lane >> 3);
          const int lc = (lane & 7) ^ ((row >> 1) & 7);
          voff[h][t] = (int)(((long)row * ld + lc * 8) * 2);
        } else {
          const int k = 2 * i + (lane >> 5);
          const int lc = (lane & 31) ^ mc_swz(k);
          voff[h][t] = (int)(((long)k * ld + lc * 8) * 2);
        }
      }
    base = (const char*)(KC ? P + (long)r0 * ld : P + r0);
    kstride = KC ? 2 : ld * 2;
  }
  // the same pieces from another tile's origin (the persistent kernel walks several tiles with one set of offsets)
  __device__ __forceinline__ void half_from(const char* org, int k0, char* lds, int h, int wave) const {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(org + (long)k0 * kstride), (short)0,
                                                                       0x7fffffff, 0x00020000);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(lds + (16 * h + 2 * wave + t) * 1024), 16,
                                               voff[h][t], 0, 0, 0);
  }
  template <bool ASM = false>
  __device__ __forceinline__ void half(int k0, char* lds, int h, int wave) const {
    if constexpr (ASM) {
#pragma unroll
      for (int t = 0; t < 2; ++t) dma_asm(base + (long)k0 * kstride, lds + (16 * h + 2 * wave + t) * 1024, voff[h][t]);
    } else {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)k0 * kstride), (short)0,
                                                                         0x7fffffff, 0x00020000);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(lds + (16 * h + 2 * wave + t) * 1024), 16,
                                                 voff[h][t], 0, 0, 0);
    }
  }
};

#ifndef CMHAR_GEMM8P_ABLATE
#define CMHAR_GEMM8P_ABLATE 0
#endif
// CMHAR_GEMM8P_BEARLY (A/B knob, two A buffers): the weight operand B of K-tile t+1 staged in phase 1 and A's lower
// half in phase 2 (the default order is the reverse: B then gets two barrier intervals of lead, A's lower half three)
#ifndef CMHAR_GEMM8P_BEARLY
#define CMHAR_GEMM8P_BEARLY 0
#endif


// The weight-gradient A operand (dYᵀ: [k][m], m contiguous) on the 8-phase schedule, staged in COLUMN halves: the
// schedule hands A's half h (rows 128h.. of the output tile) to wave group h only, so each half is its own
// [64 k][128 m] image at h * 16 KiB (256-B rows, the mc_off swizzle, whose XOR never leaves a half's 16 chunks); a
// 1 KiB DMA piece = 4 k-rows of 256 B.
struct DmaHalfM {
  const char* base;
  long kstride;
  int voff[2][2];
  __device__ __forceinline__ void init(const bf16* __restrict__ P, long ld, int c0, int wave, int lane) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k = 4 * (2 * wave + t) + (lane >> 4);
        const int lc = (lane & 15) ^ mc_swz(k);
        voff[h][t] = (int)(((long)k * ld + h * 128 + lc * 8) * 2);
      }
    base = (const char*)(P + c0);
    kstride = ld * 2;
  }
  template <bool ASM = false>
  __device__ __forceinline__ void half(int k0, char* lds, int h, int wave) const {
    if constexpr (ASM) {
#pragma unroll
      for (int t = 0; t < 2; ++t) dma_asm(base + (long)k0 * kstride, lds + h * 16384 + (2 * wave + t) * 1024, voff[h][t]);
    } else {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)k0 * kstride), (short)0,
                                                                         0x7fffffff, 0x00020000);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(lds + h * 16384 + (2 * wave + t) * 1024), 16,
                                                 voff[h][t], 0, 0, 0);
    }
  }
};

// A-operand fragment of the 8-phase kernel: K-contiguous image (frag256<true>) or DmaHalfM's column halves (the
// transposed reads of frag256<false> on 256-B rows).
template <bool A_KC>
__device__ __forceinline__ bf16x8 frag8p_a(const char* lds, int r0, int kk, int lane) {
  if (A_KC) return frag256<true>(lds, r0, kk, lane);
  const char* hb = lds + (r0 >> 7) * 16384;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int chunk = ((r0 & 127) >> 3) + (p >> 1);
  const int k = kk * 32 + 8 * g + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, hb + mc_off(k, chunk) + (p & 1) * 8));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, hb + mc_off(k + 4, chunk) + (p & 1) * 8));
  short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// A_KC = false: the weight-gradient layout (dW = dYᵀX, both operands row-contraction), split-K capable: blockIdx.z =
// K-split of klen (fp32 partial slabs at split_stride when raw_out, reduced by splitk_reduce_kernel), with the bias
// gradient Σ_k A(m,k) (Epilogue::rowsum) on the same MFMA operand fragments as gemm256_kernel; the per-output
// accumulation order (K-tile, then kk) is gemm256_kernel's, so the two kernels give identical bits.
// NA = 3: the A operand triple-buffered (three 32 KiB A images + two B images = the whole 160 KiB): A of K-tile t+2
// is staged during K-tile t (half 1 in phase 2, half 0 in phase 4) and B of t+1 in phase 1, so phase 4 waits with
// vmcnt(4) for B(t+1) and A(t+1) only — the activation stream (the HBM / MALL-bound operand) gets a whole K-tile more
// lead than the 2–4 barrier intervals (~0.3 µs) of the two-buffer schedule.  Same fragments, same MFMA order:
// identical bits.
// ngroup > 1 (forward layout only): the output tiles are walked in ngroup column groups — every tile row of group 0,
// then of group 1, … — so that the tiles an XCD runs (a contiguous band of this order, xcd_remap) share one group's
// weight columns.  A group's weight panel (≤ ~2 MiB) then stays in the XCD's 4 MiB L2 across chip rounds while the
// activation panels stream through; in row-major order every round needs the WHOLE weight (QKV 3.5 MiB, FC1 4.7 MiB),
// which does not fit beside the round's activation panels and is re-fetched from the MALL every round.
template <typename E, bool A_KC, bool B_KC, typename OutT, bool PFS = false, int NA = 2>
__global__ __launch_bounds__(NT2, 2) void gemm8p_kernel(int M, int N, int K, const bf16* __restrict__ A, long lda,
                                                        const bf16* __restrict__ B, long ldb, OutT* __restrict__ C,
                                                        long ldc, Epilogue e, int klen, long split_stride,
                                                        int raw_out, int ngroup) {
  static_assert(NA == 2 || NA == 3, "two or three A buffers");
  // transposed-read instantiations issue their DMA by inline asm (see dma_asm)
  constexpr bool kAD = CMHAR_GEMM8P_ASM_DMA && (!A_KC || !B_KC);
  constexpr bool kDirect = CMHAR_EPI_DIRECT && CMHAR_GEMM8P_ABLATE == 0 && !PFS;   // register-direct epilogue
  // ablation builds 3 / 4 / 5 (tools/debug): K loop only, without the B / A / both operand DMA inside the loop (the
  // prologue still stages the first K-tiles; later K-tiles read stale LDS)
  constexpr bool kAblNoB = CMHAR_GEMM8P_ABLATE == 3 || CMHAR_GEMM8P_ABLATE == 5;
  constexpr bool kAblNoA = CMHAR_GEMM8P_ABLATE == 4 || CMHAR_GEMM8P_ABLATE == 5;
  __shared__ __attribute__((aligned(16))) char smem[NA == 3 ? 163840 : SMEM2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = N / TN2, tiles_m = M / TM2, ntile = tiles_m * tiles_n;
  // split index folded into the XCD remap (as gemm256_kernel): one XCD runs whole splits
  const int rlin = xcd_remap(blockIdx.x + ntile * blockIdx.z, ntile * gridDim.z);
  const int bid = rlin % ntile, split = rlin / ntile;
  const int kbeg = split * klen, kend = min(K, kbeg + klen);
  int tm = bid / tiles_n, tn = bid % tiles_n;
  if (ngroup > 1) {
    const int cw = (tiles_n + ngroup - 1) / ngroup;          // group width in tiles (the last group may be narrower)
    const int gi = min(bid / (tiles_m * cw), ngroup - 1);
    const int wg = min(cw, tiles_n - gi * cw);
    const int loc = bid - gi * tiles_m * cw;
    tm = loc / wg;
    tn = gi * cw + loc % wg;
  }
  const int bm = tm * TM2, bn = tn * TN2;
  const int nk = (kend - kbeg) / TK2;   // >= 2 (host-checked)
  float* const rs_slab = raw_out ? (float*)C + (long)gridDim.z * split_stride + (long)split * M : nullptr;
  C += (long)split * split_stride;
  const bool rs = !A_KC && e.rowsum != nullptr && tn == tm % tiles_n;
  const float one8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const bf16x8 ones = pack_frag8<E>(one8);
  floatx4 accb[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  std::conditional_t<A_KC, DmaHalf<true>, DmaHalfM> da;
  DmaHalf<B_KC> db;
  da.init(A, lda, bm, wave, lane);
  db.init(B, ldb, bn, wave, lane);
  // NA = 2: buffer b = A image [256][64] at b*64 KiB, B image at b*64 KiB + 32 KiB; NA = 3: A images at (t % 3) *
  // 32 KiB, B images at 96 KiB + (t & 1) * 32 KiB
  auto abuf = [&](int t) -> char* { return NA == 3 ? smem + (t % 3) * 32768 : smem + (t & 1) * 65536; };
  auto bbuf = [&](int t) -> char* { return NA == 3 ? smem + 98304 + (t & 1) * 32768 : smem + (t & 1) * 65536 + 32768; };

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][4], b0[2][2], b1[2][2];

  // prologue: K-tile 0 whole + K-tile 1's A half 0 (NA = 3: K-tile 1's whole A); wait for tile 0
  da.template half<kAD>(kbeg, abuf(0), 0, wave);
  da.template half<kAD>(kbeg, abuf(0), 1, wave);
  db.template half<kAD>(kbeg, bbuf(0), 0, wave);
  db.template half<kAD>(kbeg, bbuf(0), 1, wave);
  da.template half<kAD>(kbeg + TK2, abuf(1), 0, wave);
  if constexpr (NA == 3) {
    da.template half<kAD>(kbeg + TK2, abuf(1), 1, wave);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one interval behind
  __builtin_amdgcn_sched_barrier(0);

#define MFMA_Q(QM, BF)                                                                                        \
  do {                                                                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_setprio(1);                                                                            \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                             \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                             \
      acc[(QM) * 4 + i][qn_ * 2 + j] = mma_ab<E, kDirect>(af[kk][i], BF[kk][j],         \
                                                                             acc[(QM) * 4 + i][qn_ * 2 + j]); \
    if (!A_KC && rs && qn_ == (QM)) /* bias gradient: each A fragment once, at its first quadrant */         \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                        \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                           \
        if (wc == ((QM) * 4 + i) >> 1) accb[i & 1] = mma16<E>(af[kk][i], ones, accb[i & 1]);                   \
    __builtin_amdgcn_s_setprio(0);                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_barrier();                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
  } while (0)
#define END_LOADS()                                                                                           \
  do {                                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_barrier();                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
  } while (0)

  for (int t = 0; t < nk; ++t) {
    const char* as = abuf(t);
    const char* bs = bbuf(t);
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    const int k1 = kbeg + (t + 1) * TK2, k2 = kbeg + (t + 2) * TK2;
    // phase 1: A0 + B0, stage A lower half of t+1 (NA = 3: both B halves of t+1); MFMA quadrant (0,0)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[kk][j] = frag256<B_KC>(bs, wc * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = frag8p_a<A_KC>(as, wr * 128 + i * 16, kk, lane);
    }
    if constexpr (NA == 3) {
      if (n1) {
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 0, wave);
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 1, wave);
      }
    } else if (CMHAR_GEMM8P_BEARLY) {
      if (n1) {
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 0, wave);
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 1, wave);
      }
    } else {
      if (n1) if (!kAblNoA) da.template half<kAD>(k1, abuf(t + 1), 1, wave);
    }
    END_LOADS();
    {
      constexpr int qn_ = 0;
      MFMA_Q(0, b0);
    }
    // phase 2: B1, stage both B halves of t+1 (NA = 3: A half 1 of t+2); quadrant (0,1)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[kk][j] = frag256<B_KC>(bs, wc * 64 + 32 + j * 16, kk, lane);
    if constexpr (NA == 3) {
      if (n2) if (!kAblNoA) da.template half<kAD>(k2, abuf(t + 2), 1, wave);
    } else if (CMHAR_GEMM8P_BEARLY) {
      if (n1) if (!kAblNoA) da.template half<kAD>(k1, abuf(t + 1), 1, wave);
    } else {
      if (n1) {
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 0, wave);
        if (!kAblNoB) db.template half<kAD>(k1, bbuf(t + 1), 1, wave);
      }
    }
    END_LOADS();
    {
      constexpr int qn_ = 1;
      MFMA_Q(0, b1);
    }
    // phase 3: A1 (its 8 reads are the phase's load work); quadrant (1,1)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = frag8p_a<A_KC>(as, wr * 128 + 64 + i * 16, kk, lane);
    END_LOADS();
    {
      constexpr int qn_ = 1;
      MFMA_Q(1, b1);
    }
    // phase 4: no reads; all of t+1 landed (own pieces), then A upper half of t+2; quadrant (1,0).  NA = 3: A half 0
    // of t+2 first, then a wait that leaves t+2's four A pieces in flight
    if constexpr (NA == 3) {
      if (n2) {
        if (!kAblNoA) da.template half<kAD>(k2, abuf(t + 2), 0, wave);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (n2) if (!kAblNoA) da.template half<kAD>(k2, abuf(t + 2), 0, wave);
    }
    END_LOADS();
    {
      constexpr int qn_ = 0;
      MFMA_Q(1, b0);
    }
  }
#undef MFMA_Q
#undef END_LOADS
  if (wr == 0) __builtin_amdgcn_s_barrier();   // re-align the groups
  if (!A_KC && rs && (lane & 15) == 0) {       // every column of a ones-product holds the row sum: lanes 0,16,32,48
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wr * 128 + (2 * wc + ii) * 16 + 4 * (lane >> 4) + r;
        if (rs_slab) rs_slab[m] = accb[ii][r];
        else e.rowsum[m] = e.rowsum_beta != 0.f ? accb[ii][r] + e.rowsum_beta * e.rowsum[m] : accb[ii][r];
      }
  }
  if constexpr (kDirect) {
    epi_direct<OutT, PFS>(e, C, ldc, raw_out ? (float*)C + (long)(bm + wr * 128) * ldc + bn + wc * 64 : nullptr, ldc,
                          bm + wr * 128, bn + wc * 64, lane, acc);
    return;
  }
  __syncthreads();
#if CMHAR_GEMM8P_ABLATE == 1 || CMHAR_GEMM8P_ABLATE >= 3   // ablation builds: K loop only, accumulators kept live
  {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) ((float*)C)[tid] = t;
    return;
  }
#endif

  // epilogue: as gemm256_kernel — per wave, two passes of 64x64 through a private LDS slab, 16-B stores
  float* T = (float*)(smem + wave * 64 * EPI2_LD * 4);
  long pld = 0;
  const OutT* const ps = PFS && sizeof(OutT) == 2 && !raw_out ? epi_stream<OutT>(e, pld) : nullptr;
  constexpr bool XP = PFS && CMHAR_EPI_PFD == 8 && CMHAR_EPI_XPASS;   // as gemm256_kernel
  uint4_t pwn[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pwn[j] = uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int cg = (lane & 7) * 8;
    const int n0 = bn + wc * 64 + cg;
    floatx4 bh[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    if (CMHAR_EPI_BIAS_HOIST && e.bias) {
      bh[0] = *(const floatx4*)(e.bias + n0);
      bh[1] = *(const floatx4*)(e.bias + n0 + 4);
    }
    auto pf = [&](int it) -> uint4_t {
      return ps ? *(const uint4_t*)(ps + (long)(bm + wr * 128 + pass * 64 + it * 8 + (lane >> 3)) * pld + n0)
                : uint4_t{0u, 0u, 0u, 0u};
    };
    constexpr int PD = CMHAR_EPI_PFD;   // row groups in flight (even, 2..8)
    uint4_t pw[PD];                      // pw[j]: the operand of row group it2 + j (static indices only)
#pragma unroll
    for (int j = 0; j < PD; ++j) pw[j] = PFS && !(XP && pass == 1) ? pf(j) : pwn[j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(i * 16 + 4 * (lane >> 4) + r) * EPI2_LD + j * 16 + (lane & 15)] = acc[pass * 4 + i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (XP && pass == 0 && ps) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pwn[j] = *(const uint4_t*)(ps + (long)(bm + wr * 128 + 64 + j * 8 + (lane >> 3)) * pld + n0);
    }
    auto row = [&](int it, uint4_t pre) __attribute__((always_inline)) {
      const int rr = it * 8 + (lane >> 3);
      const int m = bm + wr * 128 + pass * 64 + rr;
      const floatx4 lo = *(const floatx4*)&T[rr * EPI2_LD + cg], hi = *(const floatx4*)&T[rr * EPI2_LD + cg + 4];
      if (CMHAR_GEMM8P_ABLATE == 2) {   // ablation build: LDS staging + read-back, no global stores
        if (lo[0] + hi[3] == 1234.5f) ((float*)C)[tid] = lo[1];
      } else if (raw_out) {
        float* dst = (float*)C + (long)m * ldc + n0;
        *(floatx4*)dst = lo;
        *(floatx4*)(dst + 4) = hi;
      } else {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
        epilogue_store8<OutT>(e, C, ldc, m, n0, v, ps != nullptr, pre, CMHAR_EPI_BIAS_HOIST ? bh : nullptr);
      }
    };
    if constexpr (PFS) {
#pragma unroll 1
      for (int it2 = 0; it2 < 8; it2 += 2) {
        const uint4_t q0 = pw[0], q1 = pw[1];
#pragma unroll
        for (int j = 0; j + 2 < PD; ++j) pw[j] = pw[j + 2];
        if (it2 + PD < 8) {
          pw[PD - 2] = pf(it2 + PD);
          pw[PD - 1] = pf(it2 + PD + 1);
        }
        row(it2, q0);
        row(it2 + 1, q1);
      }
    } else {
#pragma unroll 2
      for (int it = 0; it < 8; ++it) row(it, pw[0]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// Epilogue of the persistent kernel (its launches: 16-bit output, bias already in the accumulators — the tile's
// MFMAs start from it —, key-column scale, GELU pair).  Lane l holds row (i*16 + (l&15)) and columns j*16 + 4(l>>4) + r
// (swapped MFMA operands); one v_permlane16_swap per register pairs blocks (2p, 2p+1) so that a lane holds 8
// consecutive columns 32p + {0,16,8,24}[l>>4] of its row, stored as one 16-B store (16 rows x 64 B per instruction).
// The s_memtime timeline (tools/debug/persist_probe.py) had the generic direct epilogue at 9.3 k / 12.2 k cycles per
// QKV tile for the two wave groups with ~84 VALU per 16 values (a wave64 VALU instruction holds its SIMD 4 cycles);
// here: 8 swaps, the scale, 8 converts and the address per 16 values, unrolled (the plain form), or one rolled
// iteration per row block with the accumulators picked by a switch (the GELU pair, whose math dominates).
__device__ __forceinline__ void swap_rows(const floatx4 (&a)[4], int p, float (&v)[8]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[2 * p][r]), __float_as_uint(a[2 * p + 1][r]),
                                                    false, false);
    v[r] = __uint_as_float(s[0]);
    v[4 + r] = __uint_as_float(s[1]);
  }
}
template <typename OutT>
__device__ __forceinline__ void epi_persist(const Epilogue& e, OutT* __restrict__ C, long ldc, int m0, int n0,
                                            int lane, const floatx4 (&acc)[8][4]) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef OutT __attribute__((ext_vector_type(2))) o2;
  typedef int __attribute__((ext_vector_type(4))) i4;
  // (the lane made opaque per tile: hoisted out of the tile loop, its 64-bit row/column bases were spilled — and the
  // scratch reload's vmcnt(0) drained the next tile's pre-issued DMA)
  int lz = lane;
  asm volatile("" : "+v"(lz));
  const int g = lz >> 4, li = lz & 15;
  const int cofs = ((g & 1) << 4) | ((g >> 1) << 3);
  const bool gp = e.act == ACT_GELU_SAVEGRAD && e.aux_out;
  const bool any_cs = e.colscale_hi > e.colscale_lo;
  f2 s2[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int col = n0 + 32 * p + cofs;   // a multiple-of-8 scale range: whole 8-column groups
    const float sc = col >= e.colscale_lo && col < e.colscale_hi ? e.colscale : 1.f;
    s2[p] = f2{sc, sc};
  }
  OutT* const c0 = C + (long)(m0 + li) * ldc + n0 + cofs;
  auto put = [&](const i4& v, OutT* dst) __attribute__((always_inline)) {
    if (CMHAR_NT_STORE) __builtin_nontemporal_store(v, (i4*)dst);
    else *(i4*)dst = v;
  };
  if (!gp) {
    // streamed operand (16-bit, this lane's 8 columns per segment): every segment's 16 B loaded up front — issued
    // after the boundary DMA, so each one's wait (counted by the compiler) leaves the stores of the earlier
    // segments in flight
    const bool mul = e.act == ACT_MULAUX;
    const OutT* const sp = mul ? (const OutT*)e.aux_in : (const OutT*)e.residual;
    const long sld = mul ? e.lda : e.ldr;
    i4 sv[16];
    if (sp) {
      const OutT* const s0 = sp + (long)(m0 + li) * sld + n0 + cofs;
#pragma unroll
      for (int c = 0; c < 16; ++c) {   // (16-B aligned: the host checks 8-element leading dimensions)
        const i4* q = (const i4*)__builtin_assume_aligned(s0 + (long)(c >> 1) * 16 * sld + 32 * (c & 1), 16);
        sv[c] = __builtin_nontemporal_load(q);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float v[8];
        swap_rows(acc[i], p, v);
        i4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f2 x = {v[2 * k], v[2 * k + 1]};
          if (any_cs) x = x * s2[p];
          if (sp) {
            // (element copied out first: a bit_cast straight off an ext-vector subscript reads element 0)
            const int w = sv[2 * i + p][k];
            const f2 t = __builtin_convertvector(__builtin_bit_cast(o2, w), f2);
            x = mul ? x * t : x + t;
          }
          o[k] = __builtin_bit_cast(int, __builtin_convertvector(x, o2));
        }
        put(o, c0 + (long)i * 16 * ldc + 32 * p);
      }
    return;
  }
  OutT* const a0 = (OutT*)e.aux_out + (long)(m0 + li) * e.ldo + n0 + cofs;
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    float v[2][8];
    switch (i) {
#define CMHAR_PICK(I) case I: swap_rows(acc[I], 0, v[0]); swap_rows(acc[I], 1, v[1]); break;
      CMHAR_PICK(0) CMHAR_PICK(1) CMHAR_PICK(2) CMHAR_PICK(3) CMHAR_PICK(4) CMHAR_PICK(5) CMHAR_PICK(6)
      default: swap_rows(acc[7], 0, v[0]); swap_rows(acc[7], 1, v[1]); break;
#undef CMHAR_PICK
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      i4 o, a;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f2 x = {v[p][2 * k], v[p][2 * k + 1]}, t;
        if (any_cs) x = x * s2[p];
        gelu_pair16x2(x, x, t);
        o[k] = __builtin_bit_cast(int, __builtin_convertvector(x, o2));
        a[k] = __builtin_bit_cast(int, __builtin_convertvector(t, o2));
      }
      put(a, a0 + (long)i * 16 * e.ldo + 32 * p);
      put(o, c0 + (long)i * 16 * ldc + 32 * p);
    }
  }
}
// The bias columns of a lane in the swapped accumulator layout (block j: columns n0 + j*16 + 4(l>>4) .. +3) — the
// persistent kernel starts each tile's accumulators from them (zeros without a bias) — read from the workgroup's LDS
// copy of the bias vector: a global load there left a pending load across the epilogue, whose wait the compiler could
// not count past the stores (it waited vmcnt(0..3) at the next tile's first MFMAs, draining the epilogue's stores)
constexpr int kPersistBiasMax = 4096;   // bias floats an LDS copy holds (N of a persistent launch, host-checked)
__device__ __forceinline__ void bias_init(const Epilogue& e, const float* lds_bias, int n0, int lane, floatx4 (&b)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (e.bias) {
    int lz = lane;                        // (opaque per call: a hoisted lane-dependent address was spilled)
    asm volatile("" : "+v"(lz));
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *(const floatx4*)(lds_bias + n0 + j * 16 + 4 * (lz >> 4));
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Persistent 8-phase forward-layout kernel (CMHAR_GEMM8P_PERSIST; whole K, no streamed epilogue operand): one
// workgroup per CU walks tiles v = blockIdx.x + G·s (G = the CU count, a multiple of 8, so that iteration s of every
// workgroup is exactly round s of the one-tile-per-workgroup launch: the same tile set per XCD at the same time).  The
// 8-phase K loop runs over the CONCATENATED K-tiles of the workgroup's tiles — the next tile's K-tile 0 (and the lower
// A half of its K-tile 1) is staged under the current tile's last K-tile exactly like any other K-tile.  At a tile
// boundary each wave, right after its last MFMA quadrant (group 0 one interval before group 1, while the other group's
// MFMAs run): (1) issues the rest of the next tile's K-tile 1 (A upper half + B) into the buffer the finished K-tile
// just released — BEFORE (2) the register-direct epilogue (epi_direct: no LDS) issues its stores.  vmcnt counts loads,
// stores and LDS-DMA in issue order (gfx9 has no separate store counter), so the K-tile-1 wait in the next tile's
// K-tile 0 is a counted `vmcnt(S)` that leaves the S epilogue memory operations of this wave in flight: the stores drain
// under the next tile's K loop instead of holding the workgroup (and its CU) until they are acknowledged, and the next
// workgroup's launch and first-K-tile latency disappear.  No inter-workgroup communication: a workgroup that is not
// resident yet just starts later.
//
// Tile claiming (sched != nullptr, CMHAR_PERSIST_DYNAMIC): instead of the fixed walk v = blockIdx + G·s, a workgroup
// claims its tiles from its XCD's counter (sched[blockIdx % 8], the XCD's contiguous chunk of the xcd_remap order) —
// one returning vector atomic of thread 0 per tile, issued one tile ahead inside K-tile 1, before that K-tile's
// vmcnt(0), and handed to the other waves through LDS.  A workgroup that starts late (its CU held by a kernel of
// another stream: the IMU branch's 32 long workgroups) then claims fewer tiles instead of finishing its fixed share
// that much later.  Every tile is computed exactly as before, so the output is the same whoever claims it.  The last
// workgroup to finish (sched[8] counts them) puts the counters back to zero for the next launch on the stream.
template <typename E, typename OutT>
__global__ __launch_bounds__(NT2, 2) void gemm8p_persist_kernel(int M, int N, int K, const bf16* __restrict__ A,
                                                                long lda, const bf16* __restrict__ B, long ldb,
                                                                OutT* __restrict__ C, long ldc, Epilogue e,
                                                                int ngroup, unsigned* sched) {
  __shared__ __attribute__((aligned(16))) char smem[131072 + kPersistBiasMax * 4 + 16];
  const int tid = threadIdx.x, lane = tid & 63, lane_ = lane;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = N / TN2, tiles_m = M / TM2, ntile = tiles_m * tiles_n;
  const int nk = K / TK2;   // even, >= 2 (host-checked; >= 4 with sched)
  float* const lds_bias = (float*)(smem + 131072);   // N <= kPersistBiasMax (host-checked)
  int* const slot = (int*)(smem + 131072 + kPersistBiasMax * 4);   // claimed tiles handed to the other waves
  if (e.bias)
    for (int c = tid * 4; c < N; c += NT2 * 4) *(floatx4*)(lds_bias + c) = *(const floatx4*)(e.bias + c);
  const int G = gridDim.x;
  // this workgroup's XCD chunk of the xcd_remap order (the tiles its XCD's counter hands out)
  const int xcd = blockIdx.x & 7, q8 = ntile >> 3, r8 = ntile & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcnt = q8 + (xcd < r8 ? 1 : 0);
  auto valid = [&](unsigned v) -> int { return v < (unsigned)xcnt ? (int)v : -1; };
  auto finish = [&]() {        // thread 0 only, after its last claim
    if (atomicAdd(sched + 8, 1u) == (unsigned)(G - 1)) {
#pragma unroll
      for (int x = 0; x < 9; ++x) atomicExch(sched + x, 0u);
    }
  };
  if (sched) {
    if (tid == 0) {   // the first two tiles in one claim (counter values only grow: if the first is past the chunk, so
      const unsigned v = atomicAdd(sched + xcd, 2u);   // is the second)
      slot[0] = valid(v);
      slot[1] = valid(v + 1);
    }
    __syncthreads();
  }
  // tile origin (rows bm, columns bn) of iteration s (static walk) or of claimed chunk index s (sched), as
  // gemm8p_kernel maps block id v
  auto tile_of = [&](int s, int& bm, int& bn) -> bool {
    int bid;
    if (sched) {
      if (s < 0) return false;
      bid = xstart + s;
    } else {
      const int v = blockIdx.x + G * s;
      if (v >= ntile) return false;
      bid = xcd_remap(v, ntile);
    }
    int tm = bid / tiles_n, tn = bid % tiles_n;
    if (ngroup > 1) {
      const int cw = (tiles_n + ngroup - 1) / ngroup;
      const int gi = min(bid / (tiles_m * cw), ngroup - 1);
      const int wg = min(cw, tiles_n - gi * cw);
      const int loc = bid - gi * tiles_m * cw;
      tm = loc / wg;
      tn = gi * cw + loc % wg;
    }
    bm = tm * TM2;
    bn = tn * TN2;
    return true;
  };
  int bm, bn, bm2 = 0, bn2 = 0;
  if (!tile_of(sched ? slot[0] : 0, bm, bn)) {
    if (sched && tid == 0) finish();
    return;
  }
  bool nxt = tile_of(sched ? slot[1] : 1, bm2, bn2);
  DmaHalf<true> da, db;
  da.init(A, lda, bm, wave, lane);
  db.init(B, ldb, bn, wave, lane);
  const char* a_cur = (const char*)(A + (long)bm * lda);
  const char* b_cur = (const char*)(B + (long)bn * ldb);
  const char* a_nxt = (const char*)(A + (long)bm2 * lda);
  const char* b_nxt = (const char*)(B + (long)bn2 * ldb);
  auto abuf = [&](int t) -> char* { return smem + (t & 1) * 65536; };
  auto bbuf = [&](int t) -> char* { return smem + (t & 1) * 65536 + 32768; };
  // K-tile t of the concatenated stream, t >= nk meaning the next tile's K-tile t - nk
  auto stage_a = [&](int t, int h) {
    if (t < nk) da.half_from(a_cur, t * TK2, abuf(t), h, wave);
    else if (nxt) da.half_from(a_nxt, (t - nk) * TK2, abuf(t), h, wave);
  };
  auto stage_b = [&](int t) {
    if (t < nk) {
      db.half_from(b_cur, t * TK2, bbuf(t), 0, wave);
      db.half_from(b_cur, t * TK2, bbuf(t), 1, wave);
    } else if (nxt) {
      db.half_from(b_nxt, (t - nk) * TK2, bbuf(t), 0, wave);
      db.half_from(b_nxt, (t - nk) * TK2, bbuf(t), 1, wave);
    }
  };

  // accumulators start from the bias (the epilogue then adds none): out = bias + Σ_k a·b, summed in that order —
  // exact on integer data, within fp32 rounding of (Σ_k a·b) + bias otherwise
  floatx4 acc[8][4], binit[4];
  if (!sched) __syncthreads();   // the LDS bias copy (with sched: the barrier above)
  bias_init(e, lds_bias, bn + wc * 64, lane, binit);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = binit[j];
  bf16x8 af[2][4], b0[2][2], b1[2][2];

  if (CMHAR_PERSIST_STAGGER > 0) {   // A/B knob: start-time stagger (quarters of the CUs of each XCD)
    const int q = (blockIdx.x >> 3) & 3;
    for (int r = 0; r < q * CMHAR_PERSIST_STAGGER; ++r) __builtin_amdgcn_s_sleep(127);
  }
  // prologue (first tile only): K-tile 0 whole + K-tile 1's A half 0, wait for K-tile 0
  stage_a(0, 0);
  stage_a(0, 1);
  stage_b(0);
  stage_a(1, 0);
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one interval behind
  __builtin_amdgcn_sched_barrier(0);

#define MFMA_QP(QM, BF)                                                                                       \
  do {                                                                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_setprio(1);                                                                            \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                             \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                             \
      acc[(QM) * 4 + i][qn_ * 2 + j] = mma_ab<E, true>(af[kk][i], BF[kk][j], acc[(QM) * 4 + i][qn_ * 2 + j]);  \
    __builtin_amdgcn_s_setprio(0);                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_barrier();                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
  } while (0)
#define END_LOADS_P()                                                                                         \
  do {                                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    __builtin_amdgcn_s_barrier();                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
  } while (0)

  // memory operations a boundary epilogue of this wave surely issues after the pre-issued K-tile-1 DMA (a lower
  // bound: vmcnt(S) must leave only operations younger than that DMA in flight) — its 16 C stores (one 16-B store per
  // row segment), plus 16 GELU' / pre-activation stores when the epilogue writes them
  const bool aux_st = e.aux_out && (e.act == ACT_GELU || e.act == ACT_GELU_SAVEGRAD);
  const int s_ops = 16 + (aux_st ? 16 : 0);
  bool pre = false;   // this tile's K-tile 1 (A upper half + B) was issued at the previous boundary
  // one K-tile of the 8-phase loop; skip: K-tile 0 of a tile whose K-tile 1 was issued at the boundary
  auto ktile = [&](int t, bool skip) __attribute__((always_inline)) {
    const char* as = abuf(t);
    const char* bs = bbuf(t);
    // the fragment addresses recomputed per K-tile from an opaque lane (hoisted out of the tile loop they held ~a dozen
    // VGPRs for the whole kernel and pushed it into scratch once tile claiming was added)
    int lane = lane_;
    asm volatile("" : "+v"(lane));
    // phase 1: A0 + B0, stage A upper half of t+1; MFMA quadrant (0,0)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[kk][j] = frag256<true>(bs, wc * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = frag8p_a<true>(as, wr * 128 + i * 16, kk, lane);
    }
    if (!skip) stage_a(t + 1, 1);
    END_LOADS_P();
    {
      constexpr int qn_ = 0;
      MFMA_QP(0, b0);
    }
    // phase 2: B1, stage both B halves of t+1; quadrant (0,1)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[kk][j] = frag256<true>(bs, wc * 64 + 32 + j * 16, kk, lane);
    if (!skip) stage_b(t + 1);
    END_LOADS_P();
    {
      constexpr int qn_ = 1;
      MFMA_QP(0, b1);
    }
    // phase 3: A1; quadrant (1,1)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = frag8p_a<true>(as, wr * 128 + 64 + i * 16, kk, lane);
    END_LOADS_P();
    {
      constexpr int qn_ = 1;
      MFMA_QP(1, b1);
    }
    // phase 4: all of t+1 landed (own pieces; after a boundary: everything but the epilogue's memory operations),
    // then A lower half of t+2; quadrant (1,0).  sched: thread 0 claims the tile after next in K-tile 1, just before
    // that K-tile's vmcnt(0), and hands it over through LDS after it (no wait of its own on the atomic's return)
    // (the atomic as inline asm: the compiler then neither waits on its return right away nor moves it to a scalar
    // register; the vmcnt(0) below retires it, and the compiler's own counted waits only over-count with it)
    unsigned claimed = ~0u;
    if (sched && t == 1 && nxt && tid == 0) {
      asm volatile("global_atomic_add %0, %1, %2, %3 sc0" : "=v"(claimed) : "v"(xcd * 4), "v"(1u), "s"(sched)
                   : "memory");
    }
    if (skip) {
      if (s_ops >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else if (CMHAR_PERSIST_ABL == 1 && t == 1) {   // ablation build: K-tile 2's wait leaves the stores in flight
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // (wrong data when the stores are not done: timing only)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (sched && t == 1 && tid == 0) {
      asm volatile("" : "+v"(claimed));   // first use of the atomic's return: after the vmcnt(0) above, not before it
      slot[2] = valid(claimed);           // (-1 when there is no next tile: nothing was claimed)
    }
    stage_a(t + 2, 0);
    END_LOADS_P();
    {
      constexpr int qn_ = 0;
      MFMA_QP(1, b0);
    }
  };
  auto stamp = [&](int s, int k) {
#if CMHAR_PERSIST_PROBE
    const unsigned long long tm = __builtin_amdgcn_s_memtime();
    if ((wave & 3) == 0 && lane == 0 && blockIdx.x < 256 && s < 12)
      g_persist_probe[((blockIdx.x * 12 + s) * 2 + wr) * 6 + k] = tm;
#endif
  };
  for (int s = 0;; ++s) {
    stamp(s, 0);
    ktile(0, pre);
    stamp(s, 1);
#pragma unroll 1
    for (int t = 1; t < nk; ++t) ktile(t, false);
    stamp(s, 2);
    // tile boundary (this wave's MFMAs of the tile are done; every read of the last K-tile's buffers has returned).
    // The groups re-align first (group 0 waits out group 1's last quadrant), so that both run their epilogues at
    // once, as the one-tile kernel does: with the ping-pong offset kept, group 1's epilogue interval followed group 0's
    // and the store phases of the two groups serialised (QKV 190 -> 224 us)
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's bias columns (LDS)
    if (nxt) bias_init(e, lds_bias, bn2 + wc * 64, lane, binit);
    if (nxt) {
      stage_a(nk + 1, 1);
      stage_b(nk + 1);
    }
    asm volatile("" ::: "memory");   // the epilogue's memory operations stay younger than that DMA (vmcnt(S) below)
    stamp(s, 3);
    if (CMHAR_PERSIST_ABL != 2)      // ablation build 2: no epilogue at all
      epi_persist<OutT>(e, C, ldc, bm + wr * 128, bn + wc * 64, lane, acc);
    else {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (sum == 1234.5f) C[tid] = (OutT)sum;
    }
    stamp(s, 4);
    if (!nxt) {
      if (sched && tid == 0) finish();
      break;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = binit[j];
    bm = bm2;
    bn = bn2;
    a_cur = a_nxt;
    b_cur = b_nxt;
    int claimed_next = -1;
    if (sched) {   // the tile after next (claimed in K-tile 1), read by inline asm: a compiler LDS read here, behind the
                   // LDS-DMA in flight, got a vmcnt(0) that drained the epilogue's stores
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(claimed_next)
                   : "v"((unsigned)(uintptr_t)(slot + 2)) : "memory");
      claimed_next = __builtin_amdgcn_readfirstlane(claimed_next);
    }
    nxt = tile_of(sched ? claimed_next : s + 2, bm2, bn2);
    a_nxt = (const char*)(A + (long)bm2 * lda);
    b_nxt = (const char*)(B + (long)bn2 * ldb);
    pre = true;
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 falls one interval behind again (as in the prologue)
    __builtin_amdgcn_sched_barrier(0);
  }
#undef MFMA_QP
#undef END_LOADS_P
}

// Tail split for a whole-K 256² GEMM whose tile count leaves the last round of the chip mostly empty: keep full
// rounds data-parallel and split the remaining tile rows along K to fill the last round.
constexpr int kCUs = 256;
struct TailSplit {
  int n_dp, n_sk, nsplit, sk_klen, tail_m0;
};
static TailSplit tail_split(int M, int N, int K) {
  TailSplit t{0, 0, 0, 0, 0};
  if (M % TM2 || N % TN2 || K % TK2) return t;
  const int tiles_n = N / TN2, ntile = (M / TM2) * tiles_n;
  if (ntile <= kCUs) return t;
  const int rem = ntile % kCUs;
  if (rem == 0 || rem * 2 > kCUs) return t;                 // last round already more than half full
  const int n_dp = (ntile / kCUs) * kCUs / tiles_n * tiles_n; // row-aligned
  const int n_tail = ntile - n_dp;
  // the split partials cost a write + read of n_tail tiles of fp32 per split: only worth it when the tail tiles'
  // K loop is long (measured on MI355X: N = 768 at K = 3072 / 2304 gains ~30 us, at K = 768 it loses ~30 us; running
  // the K = 768 tail rows as 128² tiles in a second launch instead measured neutral)
  if (K < 2048) return t;
  int s = kCUs / n_tail;
  s = min(s, K / TK2 / 4);                                    // ≥ 4 K-tiles per split
  if (s < 2) return t;
  const int klen = cdiv(cdiv(K, s), TK2) * TK2;
  t.nsplit = cdiv(K, klen);
  t.sk_klen = klen;
  t.n_dp = n_dp;
  t.n_sk = n_tail * t.nsplit;
  t.tail_m0 = n_dp / tiles_n * TM2;
  return t;
}

// 8-phase ping-pong kernel for the forward layout; CMHAR_GEMM_8P=0/1 overrides the build default (A/B measurements).
#ifndef CMHAR_GEMM_8P_DEFAULT
#define CMHAR_GEMM_8P_DEFAULT 1
#endif
static bool use_8p() {
  static const bool v = [] {
    const char* s = getenv("CMHAR_GEMM_8P");
    return s ? atoi(s) != 0 : CMHAR_GEMM_8P_DEFAULT != 0;
  }();
  return v;
}

// The dgrad layout (B row-contraction, transposed fragment reads) builds and is exact on the same kernel, but measured
// 11 % slower on FC2 dgrad and neutral elsewhere: off unless CMHAR_GEMM_8P_DGRAD=1 at build time.
#ifndef CMHAR_GEMM_8P_DGRAD
#define CMHAR_GEMM_8P_DGRAD 0
#endif
static bool use_8p_dgrad() {
  static const bool v = [] {
    const char* s = getenv("CMHAR_GEMM_8P_DGRAD");
    return s ? atoi(s) != 0 : CMHAR_GEMM_8P_DGRAD != 0;
  }();
  return v;
}

// The weight-gradient layout (both operands row-contraction, split-K, fused bias gradient) on the 8-phase schedule;
// CMHAR_GEMM_8P_WGRAD=0/1 overrides the build default (A/B measurements; the two kernels give identical bits).
#ifndef CMHAR_GEMM_8P_WGRAD_DEFAULT
#define CMHAR_GEMM_8P_WGRAD_DEFAULT 1
#endif
static bool use_8p_wgrad() {
  static const bool v = [] {
    const char* s = getenv("CMHAR_GEMM_8P_WGRAD");
    return s ? atoi(s) != 0 : CMHAR_GEMM_8P_WGRAD_DEFAULT != 0;
  }();
  return v;
}

// A-operand buffers of the 8-phase kernel (gemm8p_kernel NA): forward / dgrad layouts and the weight-gradient
// layout separately; CMHAR_GEMM8P_NA / CMHAR_GEMM8P_WGRAD_NA = 2 / 3 override the build defaults (A/B measurements;
// identical bits either way).
#ifndef CMHAR_GEMM8P_NA_DEFAULT
#define CMHAR_GEMM8P_NA_DEFAULT 2
#endif
// (weight gradients with three A buffers, round 6: 252 VGPRs, no scratch, identical bits, but QKV / FC1 / out-proj
// wgrad 177 / 222 / 76 -> 188 / 243 / 84 us and FC2 240 -> 232 in one process, bench step -1.8 %: two)
#ifndef CMHAR_GEMM8P_WGRAD_NA_DEFAULT
#define CMHAR_GEMM8P_WGRAD_NA_DEFAULT 2
#endif
static int na_knob(const char* name, int dflt) {
  const char* s = getenv(name);
  const int v = s ? atoi(s) : dflt;
  return v == 3 ? 3 : 2;
}
static int gemm8p_na(bool ak) {
  static const int fwd = na_knob("CMHAR_GEMM8P_NA", CMHAR_GEMM8P_NA_DEFAULT);
  static const int wg = na_knob("CMHAR_GEMM8P_WGRAD_NA", CMHAR_GEMM8P_WGRAD_NA_DEFAULT);
  return ak ? fwd : wg;
}

// chip rounds of 256² tiles from which a launch takes the persistent kernel (debug builds lower it)
#ifndef CMHAR_PERSIST_MIN_ROUNDS
#define CMHAR_PERSIST_MIN_ROUNDS 3
#endif
// The persistent 8-phase forward kernel (gemm8p_persist_kernel) for whole-K forward-layout launches whose epilogue
// streams no 16-bit operand; CMHAR_GEMM8P_PERSIST=0/1 overrides the build default (A/B measurements; identical bits).
#ifndef CMHAR_GEMM8P_PERSIST_DEFAULT
#define CMHAR_GEMM8P_PERSIST_DEFAULT 1
#endif
static bool use_8p_persist() {
  static const bool v = [] {
    const char* s = getenv("CMHAR_GEMM8P_PERSIST");
    return s ? atoi(s) != 0 : CMHAR_GEMM8P_PERSIST_DEFAULT != 0;
  }();
  return v;
}
// CUs of the current device (the persistent grid); 0 when it is not a multiple of 8 (the XCD round-robin the tile
// order relies on), which disables the persistent kernel
static int persist_grid() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return n % 8 == 0 ? n : 0;
}
// CMHAR_PERSIST_BALANCE = 1 (CMHAR_PERSIST_BALANCE env overrides): the persistent grid sized so that every workgroup
// runs the same number of tiles, ⌈tiles / ⌈tiles / CUs⌉⌉ rounded up to a multiple of 8 (the N = 768 launches: 588
// tiles = 2.3 chip rounds → 200 workgroups of 3 tiles instead of 256 with a 30 %-full last round), and launches from
// 2 chip rounds up take the persistent kernel — ahead of the tail split.  Round 6 (tools/debug/gemm_ab.py --epi, one
// process): out-proj forward 86.8 → 94.7 µs, FC2 forward 245.4 → 250.9, embed 115.9 → 108.5, bench step 726.1 / 727.8
// → 726.8 / 724.2 clips/s — off.  (hipBLASLt's stream-K kernel runs the out-proj shape on 196 workgroups of 3 tiles
// at 63 µs; ours does not speed up per tile with fewer CUs busy.)
#ifndef CMHAR_PERSIST_BALANCE_DEFAULT
#define CMHAR_PERSIST_BALANCE_DEFAULT 0
#endif
static bool persist_balance() {
  static const bool v = [] {
    const char* s = getenv("CMHAR_PERSIST_BALANCE");
    return s ? atoi(s) != 0 : CMHAR_PERSIST_BALANCE_DEFAULT != 0;
  }();
  return v;
}
static int persist_grid_for(int tiles) {
  static const int g = persist_grid();
  if (!persist_balance() || g == 0) return g;
  const int rounds = cdiv(tiles, g);
  return min(g, cdiv(cdiv(tiles, rounds), 8) * 8);
}
// Tile claiming for the persistent kernel (see gemm8p_persist_kernel): one counter block per (device, stream) — 8
// per-XCD counters + a finished-workgroup count, zeroed once here and by each launch's last workgroup after that.
// CMHAR_PERSIST_DYNAMIC=0: the fixed tile walk (A/B runs; identical output).
#ifndef CMHAR_PERSIST_DYNAMIC_DEFAULT
#define CMHAR_PERSIST_DYNAMIC_DEFAULT 1
#endif
static unsigned* persist_sched(hipStream_t st) {
  static const bool on = [] {
    const char* v = getenv("CMHAR_PERSIST_DYNAMIC");
    return v ? atoi(v) != 0 : CMHAR_PERSIST_DYNAMIC_DEFAULT != 0;
  }();
  if (!on) return nullptr;
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, unsigned*> blocks;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = blocks.find({dev, st});
  if (it != blocks.end()) return it->second;
  void* p = nullptr;
  if (hipMalloc(&p, 16 * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, 16 * sizeof(unsigned), st) != hipSuccess) { (void)hipFree(p); return nullptr; }
  blocks[{dev, st}] = (unsigned*)p;
  return (unsigned*)p;
}
static bool persist_ok(bool ak, bool bkc, int M, int N, int K, bool pepi) {
  // pepi: a 16-bit output and an epilogue epi_persist handles (epi_persist_ok)
  if (!(ak && bkc) || !pepi || !use_8p_persist() || !CMHAR_EPI_DIRECT) return false;
  if (N > kPersistBiasMax || N % 4) return false;             // the LDS copy of the bias
  if (K % (2 * TK2) != 0) return false;                       // an even K-tile count
  // ≥ 3 chip rounds of tiles: at 2.3 rounds (the K = 768 out-projection input gradient, 588 tiles) the persistent
  // form measured 4 % slower; from QKV's 6.9 rounds (1764 tiles) up it is faster (no relaunch, next K-tiles in flight)
  static const int g = persist_grid();
  return g > 0 && (M / TM2) * (N / TN2) >= (persist_balance() ? 2 : CMHAR_PERSIST_MIN_ROUNDS) * g;
}

// Which kernel(s) a cmhar_gemm_bf16 call launches (also exported for trace labels: cmhar_gemm_bf16_plan).
enum GemmPlan {
  PLAN_128 = 0, PLAN_256 = 1, PLAN_256_TAIL = 2, PLAN_256_SPLITK = 3, PLAN_8P = 4, PLAN_128_SPLITK = 5, PLAN_8P_SPLITK = 6,
  PLAN_8P_PERSIST = 7
};
static int gemm_plan(bool ak, bool bkc, int M, int N, int K, int splits, bool has_ws, bool rowsum,
                     bool pepi = true) {
  const bool big = M % TM2 == 0 && N % TN2 == 0 && K % TK2 == 0;
  if (!big) {
    const int klen = splits > 1 ? cdiv(cdiv(K, splits), BK) * BK : K;
    return cdiv(K, klen) > 1 ? PLAN_128_SPLITK : PLAN_128;
  }
  const int klen = splits > 1 ? cdiv(cdiv(K, splits), TK2) * TK2 : K;
  const int nsplit = cdiv(K, klen);
  // the 8-phase loop needs >= 2 K-tiles in every split (the last one included)
  const bool wgrad8p = !ak && use_8p_wgrad() && klen >= 2 * TK2 && K - (nsplit - 1) * klen >= 2 * TK2;
  if (nsplit > 1) return wgrad8p ? PLAN_8P_SPLITK : PLAN_256_SPLITK;
  if (wgrad8p) return PLAN_8P;
  if (persist_balance() && ak && use_8p() && bkc && persist_ok(ak, bkc, M, N, K, pepi)) return PLAN_8P_PERSIST;
  if (has_ws && !rowsum && tail_split(M, N, K).n_dp > 0) return PLAN_256_TAIL;   // (8-phase instead: FC2 fwd 5 % slower)
  if (ak && K >= 2 * TK2 && use_8p() && (bkc || use_8p_dgrad()))
    return persist_ok(ak, bkc, M, N, K, pepi) ? PLAN_8P_PERSIST : PLAN_8P;
  return PLAN_256;
}

// Column groups of the 8-phase forward-layout kernel (see gemm8p_kernel): two when the weight panel (N·K bf16) exceeds
// 3 MiB at K ≤ 1024 (QKV, FC1 forward, FC2's input gradient on W2ᵀ) — each activation panel is then fetched twice
// (once per group) instead of the weight once per chip round; one otherwise.  CMHAR_GEMM_NGROUP=n forces n (A/B runs).
#ifndef CMHAR_GEMM_NGROUP_DEFAULT
#define CMHAR_GEMM_NGROUP_DEFAULT 0
#endif
static int gemm8p_groups(bool ak, bool bkc, int N, int K) {
  static const int force = [] {
    const char* v = getenv("CMHAR_GEMM_NGROUP");
    return v ? atoi(v) : CMHAR_GEMM_NGROUP_DEFAULT;
  }();
  if (!ak || !bkc) return 1;
  const int tiles_n = N / TN2;
  if (force > 0) return min(force, tiles_n);
  return (2L * N * K > (3L << 20) && K <= 1024 && tiles_n >= 4) ? 2 : 1;
}

template <typename E, bool AK, bool BKc, typename OutT>
int launch(int M, int N, int K, const bf16* A, long lda, const bf16* B, long ldb, OutT* C, long ldc,
           const Epilogue& e, int splits, float* ws, hipStream_t st, int phases) {
  // phases: bit 0 = the GEMM kernel, bit 1 = the split-K / tail reduce (3 = both; the split lets a tracer time
  // the GEMM kernel alone between the two launches)
  const bool ph_gemm = phases & 1, ph_red = phases & 2;
  // triple-buffered A for the forward / dgrad layouts (7-14 % faster, tools/debug/gemm_ablate.py mode 9); the
  // weight-gradient layout (both operands row-contraction) runs out of registers with it and keeps two buffers
  constexpr int kNA = AK ? 3 : 2;
  const long ss = (long)M * N;
  if (splits > 1 && !ws) return -2;
  const bool big = M % TM2 == 0 && N % TN2 == 0 && K % TK2 == 0;
  if (e.rowsum && (AK || !big)) return -3;            // row sums only on the 256-tile weight-gradient path
  if (big) {
    int klen = K;
    if (splits > 1) klen = cdiv(cdiv(K, splits), TK2) * TK2;
    const int nsplit = cdiv(K, klen);
    dim3 grid((M / TM2) * (N / TN2), 1, nsplit);
  // epilogues with a streamed 16-bit operand run the PFS instantiation (the operand loaded two row groups ahead);
  // the others keep the plain store loop (CMHAR_EPI_PF2=0: never)
  const bool pfs = CMHAR_EPI_PF2 && sizeof(OutT) == 2 && epi_has_stream(e);
    // (the persistent epilogue moves its streamed operands with 16-B vector accesses declared aligned: operands
    // that are not 16-B aligned with 8-element leading dimensions keep the other kernels)
    const auto al16 = [](const void* p, long ld) { return !p || (((uintptr_t)p & 15) == 0 && ld % 8 == 0); };
    const bool pepi = sizeof(OutT) == 2 && epi_persist_ok(e) && al16(e.residual, e.ldr) && al16(e.aux_in, e.lda) &&
                      al16(e.aux_out, e.ldo) && al16(C, ldc);
    const int plan = gemm_plan(AK, BKc, M, N, K, splits, ws != nullptr, e.rowsum != nullptr, pepi);
    if (plan == PLAN_256_TAIL) {
      const TailSplit ts = tail_split(M, N, K);
      if (ph_gemm && pfs)
        gemm256_kernel<E, AK, BKc, OutT, 0, kNA, true><<<ts.n_dp + ts.n_sk, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc,
                                                                                      e, K, 0, 0, ws, ts.n_dp,
                                                                                      ts.sk_klen);
      else if (ph_gemm)
        gemm256_kernel<E, AK, BKc, OutT, 0, kNA><<<ts.n_dp + ts.n_sk, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, K, 0,
                                                                                0, ws, ts.n_dp, ts.sk_klen);
      const int tail_rows = M - ts.tail_m0;
      if (ph_red)
        splitk_reduce_kernel<OutT><<<reduce_blocks(tail_rows, N), 256, 0, st>>>(
            tail_rows, N, ts.nsplit, ws, (long)tail_rows * N, C, ldc, e, ts.tail_m0);
    } else if (plan == PLAN_8P) {
      const bool na3 = gemm8p_na(AK) == 3;
      const int ng = gemm8p_groups(AK, BKc, N, K);
      if (ph_gemm && pfs && na3)
        gemm8p_kernel<E, AK, BKc, OutT, true, 3><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, K, 0, 0, ng);
      else if (ph_gemm && pfs)
        gemm8p_kernel<E, AK, BKc, OutT, true><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, K, 0, 0, ng);
      else if (ph_gemm && na3)
        gemm8p_kernel<E, AK, BKc, OutT, false, 3><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, K, 0, 0, ng);
      else if (ph_gemm)
        gemm8p_kernel<E, AK, BKc, OutT><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, K, 0, 0, ng);
    } else if (plan == PLAN_8P_PERSIST) {
      if constexpr (AK && BKc && sizeof(OutT) == 2) {   // (the plan requires a 16-bit output)
        const int g = persist_grid_for((M / TM2) * (N / TN2));
        // (claiming hands the tile after next over in K-tile 1: at least 4 K-tiles per tile)
        unsigned* sched = K / TK2 >= 4 ? persist_sched(st) : nullptr;
        if (ph_gemm)
          gemm8p_persist_kernel<E, OutT><<<g, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e,
                                                            gemm8p_groups(AK, BKc, N, K), sched);
      }
    } else if (plan == PLAN_8P_SPLITK) {
      if (ph_gemm && gemm8p_na(AK) == 3)
        gemm8p_kernel<E, AK, BKc, float, false, 3><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, ws, N, e, klen, ss, 1,
                                                                         1);
      else if (ph_gemm)
        gemm8p_kernel<E, AK, BKc, float><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, ws, N, e, klen, ss, 1, 1);
      if (ph_red) splitk_reduce_kernel<OutT><<<reduce_blocks(M, N), 256, 0, st>>>(M, N, nsplit, ws, ss, C, ldc, e);
    } else if (plan == PLAN_256) {
      if (ph_gemm && pfs)
        gemm256_kernel<E, AK, BKc, OutT, 0, kNA, true><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, klen, 0, 0,
                                                                         nullptr, 0, 0);
      else if (ph_gemm)
        gemm256_kernel<E, AK, BKc, OutT, 0, kNA><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, klen, 0, 0, nullptr,
                                                                   0, 0);
    } else {
      if (ph_gemm)
        gemm256_kernel<E, AK, BKc, float, 0, kNA><<<grid, NT2, 0, st>>>(M, N, K, A, lda, B, ldb, ws, N, e, klen, ss, 1,
                                                                    nullptr, 0, 0);
      if (ph_red) splitk_reduce_kernel<OutT><<<reduce_blocks(M, N), 256, 0, st>>>(M, N, nsplit, ws, ss, C, ldc, e);
    }
    CMHAR_CHECK_LAUNCH();
    return 0;
  }
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int klen = K;
  if (splits > 1) klen = cdiv(cdiv(K, splits), BK) * BK;
  const int nsplit = cdiv(K, klen);
  dim3 grid(tiles, 1, nsplit);
  const bool full = (M % BM == 0) && (N % BN == 0) && (K % BK == 0) && (klen % BK == 0);
#define GO(BND)                                                                                               \
  do {                                                                                                        \
    if (!ph_gemm) break;                                                                                      \
    if (nsplit == 1)                                                                                          \
      gemm_bf16_kernel<E, AK, BKc, OutT, BND><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, klen, 0, 0); \
    else                                                                                                      \
      gemm_bf16_kernel<E, AK, BKc, float, BND><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, ws, N, e, klen, ss, 1); \
  } while (0)
  if (full) GO(false); else GO(true);
#undef GO
  if (nsplit > 1 && ph_red)
    splitk_reduce_kernel<OutT><<<reduce_blocks(M, N), 256, 0, st>>>(M, N, nsplit, ws, ss, C, ldc, e);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// fp32 workspace floats cmhar_gemm_bf16 can use for a whole-K (splits == 1) call: the tail-split partials, or 0.
extern "C" long cmhar_gemm_bf16_ws(int M, int N, int K) {
  const TailSplit t = tail_split(M, N, K);
  return t.n_dp > 0 ? (long)t.nsplit * (M - t.tail_m0) * N : 0;
}

// The kernel plan of a cmhar_gemm_bf16 call with these arguments (GemmPlan: 0 = 128² tile, 1 = 256² tile, 2 = 256²
// + tail split + reduce, 3 = 256² split-K + reduce, 4 = 8-phase 256², 5 = 128² split-K + reduce, 6 = 8-phase 256²
// split-K + reduce), -1 on a bad layout.
extern "C" int cmhar_gemm_bf16_plan(int layout, int M, int N, int K, int splits, int has_ws, int rowsum) {
  if (layout < 0 || layout > 2) return -1;
  return gemm_plan(layout != 2, layout == 0, M, N, K, splits, has_ws != 0, rowsum != 0);
}
#if CMHAR_PERSIST_PROBE
extern "C" int cmhar_debug_persist_probe(unsigned long long* host, long n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_persist_probe), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
// As cmhar_gemm_bf16_plan for a 16-bit output whose epilogue is (reads = 0) or is not (reads != 0) one the persistent
// kernel takes (epi_persist_ok: plain, GELU pair, × aux_in, + residual; not rowadd / beta / dropout / alpha != 1).
extern "C" int cmhar_gemm_bf16_plan2(int layout, int M, int N, int K, int splits, int has_ws, int rowsum,
                                     int reads) {
  if (layout < 0 || layout > 2) return -1;
  return gemm_plan(layout != 2, layout == 0, M, N, K, splits, has_ws != 0, rowsum != 0, reads == 0);
}

// cmhar_gemm_bf16 with a phase mask (bit 0 = GEMM kernel, bit 1 = split-K / tail reduce): phases 1 then 2 is the
// same computation as one cmhar_gemm_bf16 call, split so that a tracer can bracket the GEMM kernel alone.
extern "C" int cmhar_gemm_bf16_phased(int layout, int out_dtype, int M, int N, int K, const void* A, long lda,
                                      const void* B, long ldb, void* C, long ldc, const Epilogue* epi, int splits,
                                      void* ws, hipStream_t stream, int phases) {
  if (M <= 0 || N <= 0) return 0;
  if (phases < 1 || phases > 3) return -1;
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  float* w = (float*)ws;
  Epilogue plain{};
  plain.alpha = 1.f;
  const Epilogue& e = epi ? *epi : plain;             // NULL = the plain product
  if ((e.colscale_lo | e.colscale_hi) & 7) return -1;  // whole 8-column epilogue groups
#define DISPATCH(AK, BKc)                                                                                     \
  return out_dtype == CMHAR_BF16                                                                              \
             ? launch<bf16, AK, BKc, bf16>(M, N, K, a, lda, b, ldb, (bf16*)C, ldc, e, splits, w, stream, phases)    \
             : launch<bf16, AK, BKc, float>(M, N, K, a, lda, b, ldb, (float*)C, ldc, e, splits, w, stream, phases)
  switch (layout) {
    case 0: DISPATCH(true, true);
    case 1: DISPATCH(true, false);
    case 2: DISPATCH(false, false);
    default: return -1;
  }
#undef DISPATCH
}

// layout: 0 = NT (A K-contig, B K-contig: Y = X Wᵀ), 1 = NN (A K-contig, B N-contig: dX = dY W),
//         2 = TN (A M-contig, B N-contig: dW = dYᵀ X).  ws: fp32 workspace of splits*M*N floats when splits > 1.
extern "C" int cmhar_gemm_bf16(int layout, int out_dtype, int M, int N, int K, const void* A, long lda, const void* B,
                               long ldb, void* C, long ldc, const Epilogue* epi, int splits, void* ws,
                               hipStream_t stream) {
  return cmhar_gemm_bf16_phased(layout, out_dtype, M, N, K, A, lda, B, ldb, C, ldc, epi, splits, ws, stream, 3);
}

// fp16 operands (the fp16 inference path, BASELINE config 5): the same kernels with the fp16 MFMA, forward layout
// only (Y = X·Wᵀ, A and B K-contiguous), output fp16 or fp32.  Same arguments and return codes as cmhar_gemm_bf16.
extern "C" int cmhar_gemm_f16(int layout, int out_dtype, int M, int N, int K, const void* A, long lda, const void* B,
                              long ldb, void* C, long ldc, const Epilogue* epi, int splits, void* ws,
                              hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (layout != 0 || (out_dtype != CMHAR_F16 && out_dtype != CMHAR_F32)) return -1;
  Epilogue plain{};
  plain.alpha = 1.f;
  const Epilogue& e = epi ? *epi : plain;
  if (e.rowsum) return -3;
  if ((e.colscale_lo | e.colscale_hi) & 7) return -1;
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  return out_dtype == CMHAR_F16
             ? launch<f16, true, true, f16>(M, N, K, a, lda, b, ldb, (f16*)C, ldc, e, splits, (float*)ws, stream, 3)
             : launch<f16, true, true, float>(M, N, K, a, lda, b, ldb, (float*)C, ldc, e, splits, (float*)ws, stream, 3);
}
