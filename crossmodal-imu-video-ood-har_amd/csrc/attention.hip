// Attention for the VideoMAE blocks (third-party transformers modeling_videomae.py:209-258: softmax(QKᵀ/√d)V,
// no mask, no dropout) and for the IMU encoder's nn.MultiheadAttention (attention-prob dropout p).
//
// bf16 flash path (head dim 64, MFMA 32x32x16 bf16):
//   fwd   one wave = 32 queries, 4 waves/WG share double-buffered 64-key K/V tiles in LDS.  Scores are computed
//         transposed, Sᵀ = K·Qᵀ, so each lane owns one query row (lane&31) and the online softmax is lane-local
//         (+1 cross-half exchange); P stays in registers and is the B operand of Oᵀ = Vᵀ·Pᵀ, whose accumulator
//         again has the query on the lane, so the rescale by exp(m_old - m_new) is a per-lane scalar.
//   bwd   two kernels, no atomics: dK/dV (key-block outer: S and dP with the KEY on the lane, so their
//         accumulators feed dVᵀ += dOᵀP and dKᵀ += QᵀdS directly) and dQ (query-block outer, like fwd).
//         Row constants (-lse, -delta) are folded into the accumulators before the MFMA chains.
// fp32 path (any head dim <= 64): exact-f32 scalar kernels with the same algorithm, used by the fp32 parity mode
// and the tiny IMU attention (L = 13, d = 16), including counter-hash dropout regenerated in backward.
#include "common.h"
#include "rowops.h"

#include <atomic>
#include <cstdlib>
#include <initializer_list>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

namespace {

constexpr float LOG2E = 1.4426950408889634f;

// Raw v_exp_f32: exp2f() wraps it in denormal range fix-ups (cmp/cndmask/ldexp per element) that the softmax
// does not need — arguments are <= 0 and an underflow to 0 is the right answer.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// [64 rows][64 bf16] image, 128-B rows; 16-B chunk XOR-swizzle that is conflict-free for both the row reads
// (ds_read_b128) and the transposed reads (ds_read_b64_tr_b16) of every kernel below (tools/lds_banks.py).
__device__ __forceinline__ int att_off(int row, int chunk) {
  const int f = (((row >> 1) & 1) << 2) | ((row >> 3) & 3);
  return row * 128 + ((chunk ^ f) << 4);
}

typedef __attribute__((address_space(3))) void* att_lds_ptr;
typedef __attribute__((ext_vector_type(2))) float float2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// The same [64][64] tile image written by LDS-DMA (buffer_load_dwordx4 ... lds: global → LDS without a VGPR round
// trip, no ds_write): each wave issues 2 of the tile's 8 pieces of 1 KiB (8 rows × 128 B); the DMA's LDS destination
// is lane-linear, so the att_off XOR swizzle is applied to each lane's SOURCE chunk (an involution).  Rows at or past
// `rows_total` fall outside the buffer resource's num_records and read as zero.  Per-lane offsets are computed once; a tile costs two scalar resource updates and 2 DMA instructions.
// CMHAR_ATTN_ASM_DMA = 1: the pieces issued by inline asm (as the GEMM's dma_asm, gemm_bf16.hip): with the builtin,
// hipcc sees an LDS write in flight and puts `s_waitcnt vmcnt(0)` in front of the first transposed LDS read
// (ds_read_b64_tr_b16) that follows — in the backward kernels that drained the NEXT tile's DMA near the start of every
// tile's MFMAs.  The kernels order every DMA themselves (vmcnt waits + barriers), as with the builtin.  M0 is written
// without the compiler knowing: every LDS-DMA of this file goes through TileDma, so no compiler-generated M0 use shares
// a kernel with it.
#ifndef CMHAR_ATTN_ASM_DMA
#define CMHAR_ATTN_ASM_DMA 1
#endif
struct TileDma {
  const char* base;   // row 0 of the head slice
  long row_bytes;     // ld * 2
  long valid;         // bytes of the slice that exist: (rows_total - 1) * row_bytes + 128
  int voff[2];
  __device__ __forceinline__ void init(const bf16* __restrict__ P, long ld, int rows_total, int wave, int lane) {
    base = (const char*)P;
    row_bytes = ld * 2;
    valid = rows_total > 0 ? (long)(rows_total - 1) * row_bytes + 128 : 0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 8 * (2 * wave + t) + (lane >> 3);
      const int f = (((row >> 1) & 1) << 2) | ((row >> 3) & 3);
      voff[t] = (int)(row * row_bytes + (((lane & 7) ^ f) << 4));
    }
  }
  __device__ __forceinline__ void tile(int r0, char* lds, int wave) const {
    const long off = (long)r0 * row_bytes;
    const long left = valid - off;
    const int nrec = (int)(left > 0 ? (left < 0x7fffffff ? left : 0x7fffffff) : 0);
    if constexpr (CMHAR_ATTN_ASM_DMA) {
      const unsigned long long a = (unsigned long long)(base + off);
      uint4_t rs;
      rs[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
      rs[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) & 0xffffu;
      rs[2] = __builtin_amdgcn_readfirstlane((unsigned)nrec);
      rs[3] = 0x00020000u;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(att_lds_ptr)(lds + (2 * wave + t) * 1024));
        // (s_nop: the SALU write of M0 needs one wait state before the LDS-DMA reads it)
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" :: "s"(la), "v"(voff[t]),
                     "s"(rs) : "memory");
      }
    } else {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(base + off), (short)0, nrec, 0x00020000);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (att_lds_ptr)(lds + (2 * wave + t) * 1024), 16, voff[t], 0, 0, 0);
    }
  }
};

// Row fragment for a 32x32x16 A operand: lane holds row (r0 + lane&31), cols 16t + 8(lane>>5) .. +8.
__device__ __forceinline__ bf16x8 row_frag(const char* lds, int r0, int t, int lane) {
  return *(const bf16x8*)(lds + att_off(r0 + (lane & 31), 2 * t + (lane >> 5)));
}

// Transposed fragment: lane holds element j of column c = c0 + (lane&31) over rows
//   r0 + 16s + 8(j>>2) + 4h + (j&3)   (h = lane>>5) — the k order of an MFMA accumulator reused as operand.
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int r0, int s, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const int ch = col >> 3, hb = (col & 7) * 2;
  const int ra = r0 + 16 * s + 4 * h + q;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + att_off(ra, ch) + hb));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4_t, lds + att_off(ra + 8, ch) + hb));
  short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Accumulator registers 8s..8s+7 → 16-bit operand fragment in format E (bf16, or fp16 on the inference path).
template <typename E = bf16>
__device__ __forceinline__ bf16x8 pack8(const floatx16& a, int s) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = a[8 * s + j];
  return pack_frag8<E>(x);
}

// accumulator register r of lane-half h ↔ row index (r&3) + 8(r>>2) + 4h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float xhalf(float v) { return __shfl_xor(v, 32); }

// v[lane] and v[lane ^ 32] in every lane from ONE v_permlane32_swap (a VALU half exchange: lanes 32-63 of the first
// operand trade places with lanes 0-31 of the second) instead of a ds_bpermute round trip through the LDS
__device__ __forceinline__ float2_t half_pair(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return float2_t{__uint_as_float(r[0]), __uint_as_float(r[1])};
}
// max / sum over the lane pair (lane, lane ^ 32); the max without the canonicalising v_max hipcc puts in front of an
// fmaxf of a cross-lane value (the operands are finite scores or -inf, never NaN)
__device__ __forceinline__ float pair_max(float v) {
  const float2_t p = half_pair(v);
  float m;
  asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(p[0]), "v"(p[1]));
  return m;
}
__device__ __forceinline__ float pair_sum(float v) {
  const float2_t p = half_pair(v);
  return p[0] + p[1];
}

// Row-per-lane epilogue of a 64-column output held as two 32x32 accumulators (acc[0]: columns 0-31, acc[1]: 32-63;
// row = lane & 31, half h = lane >> 5 holds columns 8k + 4h .. + 3 of each 8-column group k): the groups are paired
// with v_permlane32_swap so that every lane holds 16 contiguous bytes — lanes 0-31 columns 8k..8k+7, lanes 32-63
// 8k+8..8k+15 of groups (k, k+1) — and the row goes out in 4 16-B stores per lane instead of 8 of 8 B
// (cdna_hip_programming.md T21: the store tail is issue-bound).  Values v·scale rounded as the 8-B form did.
template <typename E>
__device__ __forceinline__ void store_row64(E* __restrict__ row, const floatx16 (&acc)[2], float scale, int h) {
  unsigned pk[8][2];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    typedef E __attribute__((ext_vector_type(2))) e2;
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const e2 v = {(E)(acc[k >> 2][4 * (k & 3) + 2 * w] * scale), (E)(acc[k >> 2][4 * (k & 3) + 2 * w + 1] * scale)};
      pk[k][w] = __builtin_bit_cast(unsigned, v);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const auto r = __builtin_amdgcn_permlane32_swap(pk[k][w], pk[k + 1][w], false, false);
      pk[k][w] = r[0];
      pk[k + 1][w] = r[1];
    }
    *(uint4_t*)(row + 8 * k + 8 * h) = uint4_t{pk[k][0], pk[k][1], pk[k + 1][0], pk[k + 1][1]};
  }
}

__device__ __forceinline__ void stage128(const TileDma& t, int r0, char* lds, int wave) {
  t.tile(r0, lds, wave);
  t.tile(r0 + 64, lds + 8192, wave);
}

// ---------------------------------------------------------------------------------------------------------------
// ragged tails: ≤ 32 rows (queries of the forward, keys of dK/dV) past the last full block, the OTHER sequence split
// four ways — each wave takes 32 rows of every 128-row stage — and the four partials merged through the LDS.
// NBUF = 2: double-buffered 128-row stages (64 KB, the stand-alone tail kernels).  NBUF = 1: one 32 KB stage buffer
// (+1 KB), so a tail group fits the LDS of the bulk kernel's workgroup and runs INSIDE that launch — dispatched
// first, its waves latency-bound beside the bulk waves on the same CUs instead of a launch of its own with the chip
// mostly idle (attn_bwd_dkdv_bf16 `ntail`; attn_fwd_bf16 the same: CMHAR_ATTN_FOLD_FWD).
// Same arithmetic and merge order either way; the two compiled forms may still contract a multiply-add differently
// (the folded forward's tail rows measured within 1 bf16 ulp of the stand-alone kernel's, dK/dV identical).
// ---------------------------------------------------------------------------------------------------------------
template <typename E, int NBUF>
__device__ __forceinline__ void fwd_tail_group(char* smem, int H, int Lq, int Lk, int q_base, int hd, int b,
                                               const bf16* __restrict__ Q, long ldq, const bf16* __restrict__ K,
                                               long ldk, const bf16* __restrict__ V, long ldv, E* __restrict__ O,
                                               long ldo, float* __restrict__ lse, float scale) {
  // smem: NBUF × [K 128 rows 16 KB | V 16 KB]; the merge's O partials reuse the first 32 KB, its m / l the next 1 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const bf16* Kb = K + (long)b * Lk * ldk + hd * 64;
  const bf16* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * LOG2E;
  const int myq = min(q_base + (lane & 31), Lq - 1);
  bf16x8 qf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) qf[t] = *(const bf16x8*)(Q + ((long)b * Lq + myq) * ldq + hd * 64 + 16 * t + 8 * h);
  floatx16 o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int nt = (Lk + 127) / 128;
  TileDma tk, tv;
  tk.init(Kb, ldk, Lk, wave, lane);
  tv.init(Vb, ldv, Lk, wave, lane);
  stage128(tk, 0, smem, wave);
  stage128(tv, 0, smem + 16384, wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int sub = (wave >> 1) * 8192, r0 = 32 * (wave & 1);   // this wave's 32 keys of the 128-key stage
  for (int st = 0; st < nt; ++st) {
    char* Ks_ = smem + (NBUF == 2 ? (st & 1) * 32768 : 0);
    char* Vs_ = Ks_ + 16384;
    const bool more = st + 1 < nt;
    if (NBUF == 2 && more) {
      stage128(tk, (st + 1) * 128, smem + ((st + 1) & 1) * 32768, wave);
      stage128(tv, (st + 1) * 128, smem + ((st + 1) & 1) * 32768 + 16384, wave);
    }
    const int kbase = st * 128 + 32 * wave;
    if (kbase < Lk) {      // a wave with no valid key in this step skips it (its m, l, O stay untouched)
      floatx16 s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) s = mma32<E>(row_frag(Ks_ + sub, r0, t, lane), qf[t], s);
      if (kbase + 32 > Lk) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + acc_row(r, h) >= Lk) s[r] = -INFINITY;
      }
      float mt = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[r]);
      mt = fmaxf(mt, xhalf(mt)) * c;
      if (__builtin_amdgcn_ballot_w64(mt > m + 8.f) != 0) {      // lazy rescale, as attn_fwd_bf16
        const float mn = fmaxf(m, mt);
        const float alpha = fexp2(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(fmaf(s[r], c, -m));
        s[r] = p;
        l += p;
      }
      bf16x8 pb[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) pb[ss] = pack8<E>(s, ss);
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mma32<E>(tr_frag(Vs_ + sub, r0, ss, d * 32, lane), pb[ss], o[d]);
    }
    if (NBUF == 1 && more) {   // the one buffer is free once every wave is past this stage
      __syncthreads();
      stage128(tk, (st + 1) * 128, smem, wave);
      stage128(tv, (st + 1) * 128, smem + 16384, wave);
    }
    if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // merge the four key quarters: m* = max m_w, L = Σ 2^(m_w − m*) l_w, O = Σ 2^(m_w − m*) O_w / L
  float* Ow = (float*)smem;            // [4][32][64]
  float* Mw = Ow + 4 * 32 * 64;        // [4][32]
  float* Lw = Mw + 128;                // [4][32]
  const float lt = l + xhalf(l);
  const int ql = lane & 31;
  if (h == 0) { Mw[wave * 32 + ql] = m; Lw[wave * 32 + ql] = lt; }
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) Ow[(wave * 32 + ql) * 64 + d * 32 + acc_row(r, h)] = o[d][r];
  __syncthreads();
  const int qi = tid >> 3, d0 = (tid & 7) * 8;
  float mw[4], mx = -INFINITY;
#pragma unroll
  for (int w = 0; w < 4; ++w) { mw[w] = Mw[w * 32 + qi]; mx = fmaxf(mx, mw[w]); }
  float wsum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float f = fexp2(mw[w] - mx);       // a quarter that saw no key: m_w = −inf → weight 0
    wsum += f * Lw[w * 32 + qi];
    const float* src = Ow + (w * 32 + qi) * 64 + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f * src[j];
  }
  const int q = q_base + qi;
  if (q < Lq) {
    const float inv = 1.f / wsum;
    typedef E __attribute__((ext_vector_type(8))) e8;
    e8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (E)(acc[j] * inv);
    *(e8*)(O + ((long)b * Lq + q) * ldo + hd * 64 + d0) = v;
    if ((tid & 7) == 0) lse[((long)b * H + hd) * Lq + q] = mx + log2f(wsum);
  }
}

template <bool PS, int NBUF>
__device__ __forceinline__ void dkdv_tail_group(char* smem, int H, int Lq, int Lk, int k_base, int hd, int b,
                                                const bf16* __restrict__ Q, long ldq, const bf16* __restrict__ K,
                                                long ldk, const bf16* __restrict__ V, long ldv,
                                                const bf16* __restrict__ dO, long lddo, const float* __restrict__ lse,
                                                const float* __restrict__ delta, bf16* __restrict__ dK, long lddk,
                                                bf16* __restrict__ dV, long lddv, float scale, float kscale) {
  // smem: NBUF × [Q 128 rows 16 KB | dO 16 KB], then NBUF × 128 −lse/c and NBUF × 128 −δ; the merge reuses 32 KB
  float* Ls = (float*)(smem + NBUF * 32768);
  float* Ds = Ls + NBUF * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const bf16* Qb = Q + (long)b * Lq * ldq + hd * 64;
  const bf16* Gb = dO + (long)b * Lq * lddo + hd * 64;
  const float* lseb = lse + ((long)b * H + hd) * Lq;
  const float* delb = delta + ((long)b * H + hd) * Lq;
  const float c = scale * LOG2E;
  const float inv_c = 1.f / c;
  const int myk = min(k_base + (lane & 31), Lk - 1);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    kf[t] = *(const bf16x8*)(K + ((long)b * Lk + myk) * ldk + hd * 64 + 16 * t + 8 * h);
    vf[t] = *(const bf16x8*)(V + ((long)b * Lk + myk) * ldv + hd * 64 + 16 * t + 8 * h);
  }
  // (register operands retired here, before the tile loop: otherwise the compiler's wait for these loads sits inside
  // the loop, counted as if its own loads were the only memory operations in flight — with the DMA issued by inline
  // asm (CMHAR_ATTN_ASM_DMA) that stalled every tile on the next tile's DMA)
#pragma unroll
  for (int t = 0; t < 4; ++t) asm volatile("" :: "v"(kf[t]), "v"(vf[t]));
  floatx16 dk[2], dv[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[d][r] = 0.f; dv[d][r] = 0.f; }
  const int nt = (Lq + 127) / 128;
  TileDma tq, tg;
  tq.init(Qb, ldq, Lq, wave, lane);
  tg.init(Gb, lddo, Lq, wave, lane);
  float lv = 0.f, dv_ = 0.f;
  auto load = [&](int st) {
    char* buf = smem + (st % NBUF) * 32768;
    stage128(tq, st * 128, buf, wave);
    stage128(tg, st * 128, buf + 16384, wave);
    // every lane loads (clamped row; only threads < 128 store): a branch-guarded load got a vmcnt(0) right after
    // it, draining the tile DMA just issued (as the bulk kernel's load_rows)
    const int q = st * 128 + (tid & 127);
    const float lr = lseb[min(q, Lq - 1)], dr = delb[min(q, Lq - 1)];
    lv = q < Lq ? -lr * inv_c : -INFINITY;
    dv_ = q < Lq ? -dr : 0.f;
  };
  auto store_consts = [&](int st) {
    if (tid < 128) { Ls[(st % NBUF) * 128 + tid] = lv; Ds[(st % NBUF) * 128 + tid] = dv_; }
  };
  load(0);
  store_consts(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int sub = (wave >> 1) * 8192, r0 = 32 * (wave & 1);   // this wave's 32 queries of the 128-query stage
  for (int st = 0; st < nt; ++st) {
    const char* Qs_ = smem + (st % NBUF) * 32768;
    const char* Gs_ = Qs_ + 16384;
    const float* L_ = Ls + (st % NBUF) * 128 + 32 * wave;
    const float* D_ = Ds + (st % NBUF) * 128 + 32 * wave;
    const bool more = st + 1 < nt;
    if (NBUF == 2 && more) load(st + 1);
    if (st * 128 + 32 * wave < Lq) {
      floatx16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = L_[acc_row(r, h)]; dp[r] = D_[acc_row(r, h)]; }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Qs_ + sub, r0, t, lane), kf[t], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Gs_ + sub, r0, t, lane), vf[t], dp, 0, 0, 0);
      }
      bf16x8 pbv[2], dbv[2];
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float2_t pv = PS ? float2_t{fexp2(s[r]), fexp2(s[r + 1])} : float2_t{fexp2(s[r] * c), fexp2(s[r + 1] * c)};
        const float2_t dv2 = pv * float2_t{dp[r], dp[r + 1]};
        const bf16x2_t pp = __builtin_convertvector(pv, bf16x2_t);
        const bf16x2_t dd = __builtin_convertvector(dv2, bf16x2_t);
        pbv[r >> 3][r & 7] = pp[0];
        pbv[r >> 3][(r & 7) + 1] = pp[1];
        dbv[r >> 3][r & 7] = dd[0];
        dbv[r >> 3][(r & 7) + 1] = dd[1];
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Gs_ + sub, r0, ss, d * 32, lane), pbv[ss], dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qs_ + sub, r0, ss, d * 32, lane), dbv[ss], dk[d], 0, 0, 0);
        }
    }
    if (more) {
      if (NBUF == 1) {   // the one buffer (and its row constants) is free once every wave is past this stage
        __syncthreads();
        load(st + 1);
      }
      store_consts(st + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  // sum the four query quarters' partials, dK then dV through one 32 KB [4][32][64] fp32 image
  float* W = (float*)smem;
  const int kl = lane & 31;
  const int ki = tid >> 3, d0 = (tid & 7) * 8;
  const int key = k_base + ki;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const floatx16* part = pass == 0 ? dk : dv;
    if (pass == 1) __syncthreads();   // the dK sums are read out
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) W[(wave * 32 + kl) * 64 + d * 32 + acc_row(r, h)] = part[d][r];
    __syncthreads();
    if (key < Lk) {
      const float f = pass == 0 ? kscale : 1.f;
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float sum = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) sum += W[(w * 32 + ki) * 64 + d0 + j];
        a[j] = (bf16)(sum * f);
      }
      bf16* dst = pass == 0 ? dK + ((long)b * Lk + key) * lddk : dV + ((long)b * Lk + key) * lddv;
      *(bf16x8*)(dst + hd * 64 + d0) = a;
    }
  }
}

// (block, head, batch) of a bulk kernel's workgroup on a (nb + ntail, H, B) grid whose first ntail·H·B linear ids
// (dispatched first) are tail groups: true for a tail group (bi.blk = its group within the head).  Both index spaces
// are XCD-remapped as flash_block, so with ntail·H·B and nb·H·B multiples of 8 a head's tail group runs on the XCD
// of its bulk blocks.  ntail = 0: flash_block.
__device__ __forceinline__ bool tail_block(int ntail, int H, BlkIdx& bi) {
  const int nx = gridDim.x, nyz = gridDim.y * gridDim.z;
  const int lin = blockIdx.x + nx * (blockIdx.y + gridDim.y * blockIdx.z);
  const int tails = ntail * nyz;
  if (lin < tails) {
    const int rt = xcd_remap(lin, tails), bh = rt / ntail;
    bi = {rt % ntail, bh % H, bh / H};
    return true;
  }
  const int nb = nx - ntail, r = xcd_remap(lin - tails, nb * nyz), bh = r / nb;
  bi = {r % nb, bh % H, bh / H};
  return false;
}

// CMHAR_ATTN_PRIO = 1: raise the wave's issue priority over each MFMA chain (as the GEMM's MFMA_Q) so the co-resident
// waves' softmax / exp VALU work fills the matrix pipe's gaps instead of delaying the chain (A/B knob)
// CMHAR_ATTN_ABL_NODMA: see attn_bwd_dq_bf16
#ifndef CMHAR_ATTN_ABL_NODMA
#define CMHAR_ATTN_ABL_NODMA 0
#endif
// CMHAR_ATTN_DMA_POS (backward kernels, A/B knob): where a tile's DMA for the next tile is issued — 0 at the tile's
// start, 1 after the first block's score / dP MFMA chain (the pieces then issue while those MFMAs drain), 2 split:
// the first operand's pieces at the start, the second's after that chain.  Round 6, one process
// (tools/debug/attn_ab.py, backward µs per layer): 878.2 / 944.2 / 908.9 — the tile start stays.  For scale, the
// in-loop DMA removed altogether (CMHAR_ATTN_ABL_NODMA, stale tiles): dK/dV −52 µs, dQ −45 µs of ~870.
#ifndef CMHAR_ATTN_DMA_POS
#define CMHAR_ATTN_DMA_POS 0
#endif
#ifndef CMHAR_ATTN_PRIO
#define CMHAR_ATTN_PRIO 0
#endif
#define PRIO_HI() do { if (CMHAR_ATTN_PRIO) __builtin_amdgcn_s_setprio(1); } while (0)
#define PRIO_LO() do { if (CMHAR_ATTN_PRIO) __builtin_amdgcn_s_setprio(0); } while (0)

// ---------------------------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------------------------
// QB q-blocks of 32 rows per wave (QB = 2: 64 rows): every K row fragment and V transposed fragment read from
// LDS feeds QB MFMA chains, so LDS read traffic per MFMA is 1/QB of the one-block form (at QB = 1 the reads
// alone saturate the CU's 128 B/clk LDS port at the MFMA rate).  A workgroup = 4 waves = 128·QB queries starting
// at q_base; K/V tiles of 64 keys are register-staged into a double-buffered LDS pair (issue early, write late).
// E: the 16-bit number format of Q/K/V/O (bf16 training path; fp16 for the fp16 inference path).
// Forward per 32-key half at 3 waves per SIMD (168 VGPRs): 4 % faster than scoring whole 64-key tiles at 2 waves
// per SIMD (tools/debug/attn_ab.py; the lazy-rescale points move, so not bit-identical to that form).  One launch
// with the last 256-query workgroup of each head partly idle instead of the 128-query tail launch: 1 % slower.
// CMHAR_ATTN_LSUM_MFMA = 1: the softmax row sum l of each 32-key half is taken on the matrix pipe as ones·Pᵀ over the
// bf16 P the PV product consumes (two extra MFMAs per q-block and half, into the dead score accumulators) instead of
// 16 VALU adds per lane: the forward is VALU-issue bound beside its MFMAs (exp, fma, add, max, cvt per score at head
// dim 64), the matrix pipe is not.  l is then the sum of the rounded weights O's numerator uses.
#ifndef CMHAR_ATTN_LSUM_MFMA
#define CMHAR_ATTN_LSUM_MFMA 1
#endif
#ifndef CMHAR_ATTN_FWD_ONE_LAUNCH
#define CMHAR_ATTN_FWD_ONE_LAUNCH 0
#endif
// OPT (optimistic running max, the default bulk launch; CMHAR_ATTN_FWD_OPT=0 at run time: one exact launch): after a
// row's first 32 keys the running max m is frozen — no half-tile max, no rescale (16 max + a lane swap per q-block
// and half: ~12 % of the VALU issue the forward is bound on).  The weights p = 2^(c·s − m) are then ≤ 2^64 for every
// row whose later scores stay within 64 (log2 units) of its first keys' max; a row past that shows as a half-tile sum
// above 2^64 (or not finite) on the MFMA row sum, its workgroup sets flag[wg], and a second launch of the exact
// kernel (gate = flag) recomputes exactly the flagged workgroups (the others return at once) and clears their flags.
// p ≤ 2^64 keeps l and O (fp32) far from overflow and bf16 P at full relative precision at any scale, so the result
// is as accurate as the lazy-rescale form, not bit-identical to it (other weight scales); lse = m + log2 l is exact
// either way.  Round 6 (tools/debug/attn_ab.py): 336.6 -> 289.1 us per layer (the optimistic kernel alone).
#ifndef CMHAR_ATTN_FWD_OPT
#define CMHAR_ATTN_FWD_OPT 1
#endif
template <typename E, int QB, bool OPT = false>
__global__ __launch_bounds__(256, 3) void attn_fwd_bf16(int H, int Lq, int Lk, int q_base, const bf16* __restrict__ Q,
                                                        long ldq, const bf16* __restrict__ K, long ldk,
                                                        const bf16* __restrict__ V, long ldv, E* __restrict__ O,
                                                        long ldo, float* __restrict__ lse, float scale,
                                                        int ntail, int q_tail0, int* __restrict__ flag) {
  static_assert(!OPT || CMHAR_ATTN_LSUM_MFMA, "the optimistic forward checks the MFMA row sums");
  __shared__ __attribute__((aligned(16))) char smem[4 * 8192 + 1024];   // +1 KB: a folded tail group's merge
#define Ks(buf) (smem + 8192 * (buf))
#define Vs(buf) (smem + 16384 + 8192 * (buf))
  const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  // exact kernel with a gate (the optimistic launch's flags): only the flagged workgroups run
  if (!OPT && flag && flag[wg] == 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  BlkIdx bi;
  if (tail_block(ntail, H, bi)) {   // ntail > 0: this workgroup is the 32-query tail group bi.blk of its head
    fwd_tail_group<E, 1>(smem, H, Lq, Lk, q_tail0 + 32 * bi.blk, bi.hd, bi.b, Q, ldq, K, ldk, V, ldv, O, ldo, lse,
                         scale);
    return;
  }
  const int hd = bi.hd, b = bi.b;
  const int q0 = q_base + bi.blk * (128 * QB) + wave * (32 * QB);
  const bf16* Qb = Q + (long)b * Lq * ldq + hd * 64;
  const bf16* Kb = K + (long)b * Lk * ldk + hd * 64;
  const bf16* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * LOG2E;

  bf16x8 qf[QB][4];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int myq = min(q0 + 32 * j + (lane & 31), Lq - 1);
#pragma unroll
    for (int t = 0; t < 4; ++t) qf[j][t] = *(const bf16x8*)(Qb + (long)myq * ldq + 16 * t + 8 * h);
  }
  // (register operands retired here, before the tile loop: otherwise the compiler's wait for these loads sits inside
  // the loop, counted as if its own loads were the only memory operations in flight — with the DMA issued by inline
  // asm (CMHAR_ATTN_ASM_DMA) that stalled every tile on the next tile's DMA)
#pragma unroll
  for (int j = 0; j < QB; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) asm volatile("" :: "v"(qf[j][t]));
  floatx16 o[QB][2];
#pragma unroll
  for (int j = 0; j < QB; ++j)
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[j][d][r] = 0.f;
  float m[QB], l[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) { m[j] = -INFINITY; l[j] = 0.f; }
  bool bad = false;   // OPT: a row of this lane left the optimistic range

  const int nt = (Lk + 63) / 64;
  TileDma tk, tv;
  tk.init(Kb, ldk, Lk, wave, lane);
  tv.init(Vb, ldv, Lk, wave, lane);
  tk.tile(0, Ks(0), wave);
  tv.tile(0, Vs(0), wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // A wave whose queries all lie past Lq (the ragged last workgroup of a head) still helps stage K/V tiles and
  // joins every barrier, but issues no MFMA / softmax work: its SIMD's matrix pipe goes to the co-resident waves.
  const bool active = q0 < Lq;
  // row-sum selector (CMHAR_ATTN_LSUM_MFMA): as a 16x16x32 A fragment, lane l is row l & 15, k-group l >> 4; ones
  // where the row's query half ((row >> 2) & 1) matches the k-group's ((l >> 4) & 1), zeros elsewhere
  const float sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
  const float sel8[8] = {sel, sel, sel, sel, sel, sel, sel, sel};
  const bf16x8 lsel = pack_frag8<E>(sel8);
  // One K/V tile; the LDS buffer index is a compile-time constant (the loop below runs the tiles in pairs), so
  // every LDS address folds into the ds_read immediate offsets instead of a v_add per read.
  auto tile = [&](auto CUR, int kt) __attribute__((always_inline)) {
    constexpr int cur = decltype(CUR)::value;
    const bool more = kt + 1 < nt;
    // Per 32-key half (kb): Sᵀ for every q-block (each K fragment read once, used QB times), its softmax, then
    // Oᵀ += Vᵀ·Pᵀ for that half — only one half's scores are live (32 fewer VGPRs than scoring the whole 64-key
    // tile first), which lets QB = 2 run at 3 waves per SIMD.
    if (more) {   // next tile DMA'd into the other buffer under this tile's math
      tk.tile((kt + 1) * 64, Ks(cur ^ 1), wave);
      tv.tile((kt + 1) * 64, Vs(cur ^ 1), wave);
    }
    if (active) {
      const int kbase = kt * 64;
#pragma unroll 1
      for (int kb = 0; kb < 2; ++kb) {
        floatx16 s[QB];
#pragma unroll
        for (int j = 0; j < QB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[j][r] = 0.f;
        PRIO_HI();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 kf = row_frag(Ks(cur), kb * 32, t, lane);
#pragma unroll
          for (int j = 0; j < QB; ++j) s[j] = mma32<E>(kf, qf[j][t], s[j]);
        }
        PRIO_LO();
        if (kbase + kb * 32 + 32 > Lk) {   // ragged last half-tile only (wave-uniform branch)
#pragma unroll
          for (int j = 0; j < QB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kbase + kb * 32 + acc_row(r, h) >= Lk) s[j][r] = -INFINITY;
        }
        bf16x8 pb[QB][2];
#pragma unroll
        for (int j = 0; j < QB; ++j) {
          if (!OPT || kbase + kb == 0) {
          float mt = -INFINITY;
#pragma unroll
          for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[j][r]);
          mt = pair_max(mt) * c;
          // Lazy rescale: the running max m only moves (and O, l are rescaled) when some row's half-tile max
          // exceeds it by more than 8 (log2 units), so p = exp2(c·s − m) ≤ 2^8 stays well inside fp32/bf16 range;
          // with the row maxima settling after the first key tiles this skips ~all rescales.  (Seeding the S
          // accumulators with −m instead of the fma below: the seed costs 16 v_mov per block, the same issue slots.)
          if (__builtin_amdgcn_ballot_w64(mt > m[j] + 8.f) != 0) {
            const float mn = fmaxf(m[j], mt);
            const float alpha = fexp2(m[j] - mn);
            m[j] = mn;
            l[j] *= alpha;
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
              for (int r = 0; r < 16; ++r) o[j][d][r] *= alpha;
          }
          }
          const float mn = m[j];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fexp2(fmaf(s[j][r], c, -mn));
            s[j][r] = p;
            if (!CMHAR_ATTN_LSUM_MFMA) l[j] += p;
          }
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) pb[j][ss] = pack8<E>(s[j], ss);
          if (CMHAR_ATTN_LSUM_MFMA) {
            // Σ_k P[q, k] over the half on a 16x16x32 MFMA: read as that shape's B operand, lane l's fragment is column
            // n = l & 15 with k-group l >> 4, i.e. query n (k-groups 0, 2) or n + 16 (k-groups 1, 3) of the 16 keys of
            // chunk ss; the A fragment `lsel` selects, for the rows a lane's accumulator holds (4·(l >> 4) .. +3),
            // the k-groups of that lane's own query — so every lane receives its query's sum (4 equal values)
            floatx4 ls = mma16<E>(lsel, pb[j][0], floatx4{0.f, 0.f, 0.f, 0.f});
            ls = mma16<E>(lsel, pb[j][1], ls);
            l[j] += ls[0];
            if (OPT) bad = bad || !(ls[0] <= 0x1p64f);
          }
        }
        PRIO_HI();
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const bf16x8 vf = tr_frag(Vs(cur), kb * 32, ss, d * 32, lane);
#pragma unroll
            for (int j = 0; j < QB; ++j) o[j][d] = mma32<E>(vf, pb[j][ss], o[j][d]);
          }
        PRIO_LO();
      }
    }
    if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own pieces of the next tile landed
    __syncthreads();
  };
  for (int kt = 0; kt < nt; kt += 2) {
    tile(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nt) tile(std::integral_constant<int, 1>{}, kt + 1);
  }
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const float lj = CMHAR_ATTN_LSUM_MFMA ? l[j] : pair_sum(l[j]);   // the MFMA row sum covers both lane halves' keys
    const float inv = 1.f / lj;
    const int q = q0 + 32 * j + (lane & 31);
    if (q < Lq) {
      store_row64<E>(O + ((long)b * Lq + q) * ldo + hd * 64, o[j], inv, h);
      if (h == 0) lse[((long)b * H + hd) * Lq + q] = m[j] + log2f(lj);   // log2-domain LSE of (scale*log2e)*s
    }
  }
  if (OPT) {
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) flag[wg] = 1;   // the exact launch redoes this workgroup
  } else if (flag && tid == 0) {
    flag[wg] = 0;   // gated rerun done (every wave read the flag before the tile loop's barriers)
  }
}

// dK, dV: one wave = 32 keys (K, V fragments in registers as B operands), q tiles of 64 staged in LDS.
// Three waves per SIMD for the dK/dV kernel (168 VGPRs, 12 B/lane spilled): its LDS-DMA staging freed the 64
// register-staged tile VGPRs; measured 4-7 % faster than two waves per SIMD (tools/debug/attn_ab.py)
// PS (pre-scaled keys): K holds bf16(scale·log2e·K) written by the QKV GEMM's epilogue (CmharEpilogue.colscale) and
// the launch passes scale = 1/log2e, so c = 1 and p = exp2(acc) needs no multiply per score (−6 % backward time:
// the kernels are VALU-issue bound beside their MFMAs); kscale is the dK output factor (the true softmax scale, so
// dK is the gradient of the unscaled key and the QKV backward is unchanged).
// CMHAR_ATTN_DKDV_PIPE = 1 (A/B knob): the tile's two 32-query blocks software-pipelined — block 1's S / dP MFMA
// chains issued right after block 0's, ahead of block 0's exp / dS VALU, which then runs while the matrix pipe works
// through block 1's chains (and block 1's VALU beside block 0's dV / dK MFMAs); both blocks' S / dP live at once, so
// two waves per SIMD (210 VGPRs).  Same operations per element in the same order: identical bits.  Round 6
// (tools/debug/attn_ab.py): backward 858.2 -> 897.9 us per layer — three waves per SIMD interleave better than the
// explicit pipeline at two; off.
#ifndef CMHAR_ATTN_DKDV_PIPE
#define CMHAR_ATTN_DKDV_PIPE 0
#endif
template <bool PS = false>
__global__ __launch_bounds__(256, CMHAR_ATTN_DKDV_PIPE ? 2 : 3) void attn_bwd_dkdv_bf16(int H, int Lq, int Lk, int k_base,
                                                             const bf16* __restrict__ Q,
                                                             long ldq, const bf16* __restrict__ K, long ldk,
                                                             const bf16* __restrict__ V, long ldv,
                                                             const bf16* __restrict__ dO, long lddo,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta, bf16* __restrict__ dK,
                                                             long lddk, bf16* __restrict__ dV, long lddv, float scale,
                                                             float kscale, int ntail, int k_tail0) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 8192 + 2 * 2 * 64 * 4];
#define Qs(buf) (smem + 8192 * (buf))
#define Gs(buf) (smem + 16384 + 8192 * (buf))
  float* Ls = (float*)(smem + 32768);          // [2][64] lse
  float* Ds = Ls + 128;                         // [2][64] delta
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  BlkIdx bi;
  if (tail_block(ntail, H, bi)) {   // ntail > 0: the 32-key tail group bi.blk of its head (same 33 KB of LDS)
    dkdv_tail_group<PS, 1>(smem, H, Lq, Lk, k_tail0 + 32 * bi.blk, bi.hd, bi.b, Q, ldq, K, ldk, V, ldv, dO, lddo, lse,
                           delta, dK, lddk, dV, lddv, scale, kscale);
    return;
  }
  const int hd = bi.hd, b = bi.b;
  const int k0 = k_base + bi.blk * 128 + wave * 32;
  const bf16* Qb = Q + (long)b * Lq * ldq + hd * 64;
  const bf16* Gb = dO + (long)b * Lq * lddo + hd * 64;
  const float* lseb = lse + ((long)b * H + hd) * Lq;
  const float* delb = delta + ((long)b * H + hd) * Lq;
  const float c = scale * LOG2E;
  const float inv_c = 1.f / c;

  const int myk = min(k0 + (lane & 31), Lk - 1);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    kf[t] = *(const bf16x8*)(K + ((long)b * Lk + myk) * ldk + hd * 64 + 16 * t + 8 * h);
    vf[t] = *(const bf16x8*)(V + ((long)b * Lk + myk) * ldv + hd * 64 + 16 * t + 8 * h);
  }
  // (register operands retired here, before the tile loop: otherwise the compiler's wait for these loads sits inside
  // the loop, counted as if its own loads were the only memory operations in flight — with the DMA issued by inline
  // asm (CMHAR_ATTN_ASM_DMA) that stalled every tile on the next tile's DMA)
#pragma unroll
  for (int t = 0; t < 4; ++t) asm volatile("" :: "v"(kf[t]), "v"(vf[t]));
  floatx16 dk[2], dv[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[d][r] = 0.f; dv[d][r] = 0.f; }

  const int nt = (Lq + 63) / 64;
  TileDma tq, tg;            // Q / dO tiles by LDS-DMA (see TileDma)
  tq.init(Qb, ldq, Lq, wave, lane);
  tg.init(Gb, lddo, Lq, wave, lane);
  float lv = 0.f, dv_ = 0.f;
  int lq = 0;
  // row constants, staged pre-negated (and -lse pre-divided by c) as accumulator seeds.  Every lane loads (no branch
  // around the loads: hipcc waited vmcnt(0) right after a branch-guarded load, draining the tile DMA just issued)
  auto load_q = [&](int qt, char* qs) { tq.tile(qt * 64, qs, wave); };
  auto load_g = [&](int qt, char* gs) {
    tg.tile(qt * 64, gs, wave);
    lq = qt * 64 + lane;
    lv = lseb[min(lq, Lq - 1)];
    dv_ = delb[min(lq, Lq - 1)];
  };
  auto load_rows = [&](int qt, char* qs, char* gs) {
    load_q(qt, qs);
    load_g(qt, gs);
  };
  auto store_rows = [&](int buf) {
    if (tid < 64) {
      Ls[buf * 64 + tid] = lq < Lq ? -lv * inv_c : -INFINITY;
      Ds[buf * 64 + tid] = lq < Lq ? -dv_ : 0.f;
    }
  };
  load_rows(0, Qs(0), Gs(0));
  store_rows(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bool active = k0 < Lk;      // waves past the last key only stage tiles and join barriers (see forward)
  // one tile per call, LDS buffer index a compile-time constant (tiles run in pairs): LDS addresses fold into
  // the ds_read immediate offsets
  auto tile = [&](auto CUR, int qt) __attribute__((always_inline)) {
    constexpr int cur = decltype(CUR)::value;
    const bool more = qt + 1 < nt && !(CMHAR_ATTN_ABL_NODMA & 1);
    constexpr int pos = CMHAR_ATTN_DMA_POS;
    if (more && (pos == 0 || !active)) load_rows(qt + 1, Qs(cur ^ 1), Gs(cur ^ 1));
    else if (more && pos == 2) load_q(qt + 1, Qs(cur ^ 1));
    const float* L_ = Ls + cur * 64;
    const float* D_ = Ds + cur * 64;
    if (CMHAR_ATTN_DKDV_PIPE && active) {
      floatx16 s[2], dp[2];
      auto chain = [&](int qb) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = qb * 32 + acc_row(r, h);
          s[qb][r] = L_[q];
          dp[qb][r] = D_[q];
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Qs(cur), qb * 32, t, lane), kf[t], s[qb], 0, 0, 0);
          dp[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Gs(cur), qb * 32, t, lane), vf[t], dp[qb], 0, 0, 0);
        }
      };
      auto finish_block = [&](int qb) __attribute__((always_inline)) {
        bf16x8 pbv[2], dbv[2];
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const float2_t pv = PS ? float2_t{fexp2(s[qb][r]), fexp2(s[qb][r + 1])}
                                 : float2_t{fexp2(s[qb][r] * c), fexp2(s[qb][r + 1] * c)};
          const float2_t dv2 = pv * float2_t{dp[qb][r], dp[qb][r + 1]};
          const bf16x2_t pp = __builtin_convertvector(pv, bf16x2_t);
          const bf16x2_t dd = __builtin_convertvector(dv2, bf16x2_t);
          pbv[r >> 3][r & 7] = pp[0];
          pbv[r >> 3][(r & 7) + 1] = pp[1];
          dbv[r >> 3][r & 7] = dd[0];
          dbv[r >> 3][(r & 7) + 1] = dd[1];
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const bf16x8 pb = pbv[ss], db = dbv[ss];
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Gs(cur), qb * 32, ss, d * 32, lane), pb, dv[d], 0, 0, 0);
            dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qs(cur), qb * 32, ss, d * 32, lane), db, dk[d], 0, 0, 0);
          }
        }
      };
      chain(0);
      __builtin_amdgcn_sched_barrier(0);
      chain(1);
      __builtin_amdgcn_sched_barrier(0);
      finish_block(0);
      __builtin_amdgcn_sched_barrier(0);
      finish_block(1);
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      if (!active || CMHAR_ATTN_DKDV_PIPE) break;
      // S = Q·Kᵀ (key on lane), pre-loaded with -lse/c so that p = exp2(c*acc)
      floatx16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qb * 32 + acc_row(r, h);
        s[r] = L_[q];
        dp[r] = D_[q];
      }
      PRIO_HI();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Qs(cur), qb * 32, t, lane), kf[t], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Gs(cur), qb * 32, t, lane), vf[t], dp, 0, 0, 0);
      }
      PRIO_LO();
      if (pos != 0 && qb == 0 && more) {
        __builtin_amdgcn_sched_barrier(0);
        if (pos == 1) load_rows(qt + 1, Qs(cur ^ 1), Gs(cur ^ 1));
        else load_g(qt + 1, Gs(cur ^ 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      // p = exp2(c·s), dS = P ∘ (dP − δ), then both packed to bf16 — written in aligned register pairs (one
      // v_pk_mul_f32 + one v_cvt_pk_bf16_f32 per pair; element-wise, the compiler paired (1,2),(3,4),... and spent
      // v_mov / v_alignbit / v_perm re-pairing them for the packs; the backward got 3 % faster, bit-identical.  The
      // same rewrite of the forward's softmax measured 5 % slower and is not used)
      bf16x8 pbv[2], dbv[2];
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float2_t pv = PS ? float2_t{fexp2(s[r]), fexp2(s[r + 1])} : float2_t{fexp2(s[r] * c), fexp2(s[r + 1] * c)};
        const float2_t dv2 = pv * float2_t{dp[r], dp[r + 1]};
        const bf16x2_t pp = __builtin_convertvector(pv, bf16x2_t);
        const bf16x2_t dd = __builtin_convertvector(dv2, bf16x2_t);
        pbv[r >> 3][r & 7] = pp[0];
        pbv[r >> 3][(r & 7) + 1] = pp[1];
        dbv[r >> 3][r & 7] = dd[0];
        dbv[r >> 3][(r & 7) + 1] = dd[1];
      }
      PRIO_HI();
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pb = pbv[ss], db = dbv[ss];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Gs(cur), qb * 32, ss, d * 32, lane), pb, dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qs(cur), qb * 32, ss, d * 32, lane), db, dk[d], 0, 0, 0);
        }
      }
      PRIO_LO();
    }
    if (more) {
      store_rows(cur ^ 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own DMA pieces of the next tile landed
    }
    __syncthreads();
  };
  for (int qt = 0; qt < nt; qt += 2) {
    tile(std::integral_constant<int, 0>{}, qt);
    if (qt + 1 < nt) tile(std::integral_constant<int, 1>{}, qt + 1);
  }
  const int key = k0 + (lane & 31);
  if (key < Lk) {
    store_row64<bf16>(dK + ((long)b * Lk + key) * lddk + hd * 64, dk, kscale, h);
    store_row64<bf16>(dV + ((long)b * Lk + key) * lddv + hd * 64, dv, 1.f, h);
  }
}

// dQ: one wave = QB blocks of 32 queries (Q, dO fragments in registers), K/V tiles of 64 keys in LDS.  With QB = 2
// every K / V row fragment and K transposed fragment read from LDS feeds two MFMA chains: the kernel's LDS read
// traffic per MFMA halves (at QB = 1 the 4 waves' reads of the shared K/V tiles took as many LDS cycles as the MFMAs
// took matrix-pipe cycles).  A workgroup = 4 waves = 128·QB queries starting at q_base.
// δ = rowsum(dO ∘ O) is computed here from the query rows this wave owns anyway (no separate pass over O and dO)
// and written for the dK/dV kernel, which runs after this one on the same stream.
// Three waves per SIMD for dQ: with the fragments read just before their MFMAs (not hoisted per key block) the
// kernel fits 168 VGPRs without spilling; measured 7 % faster than two waves per SIMD
// CMHAR_ATTN_DQ_NBUF = 3: K/V tiles triple-buffered (48 KiB per workgroup, three per CU): tile kt+2's DMA is issued at
// the start of tile kt and the end-of-tile wait leaves it in flight (vmcnt(4)), two tiles of lead instead of one.
// Measured (round 6, attn_ab.py): backward 866.5 → 881.4 µs per layer — the staging is not latency-bound; off.
// CMHAR_ATTN_ABL_NODMA (ablation builds, tools/debug; bit 0 dK/dV, bit 1 dQ): the in-loop tile DMA skipped —
// later tiles read stale LDS — to price the staging stream.
#ifndef CMHAR_ATTN_DQ_NBUF
#define CMHAR_ATTN_DQ_NBUF 2
#endif
template <int QB, bool PS = false>
__global__ __launch_bounds__(256, QB == 1 ? 3 : 2) void attn_bwd_dq_bf16(int H, int Lq, int Lk, int q_base,
                                                           const bf16* __restrict__ Q, long ldq,
                                                           const bf16* __restrict__ K, long ldk,
                                                           const bf16* __restrict__ V, long ldv,
                                                           const bf16* __restrict__ O, long ldo,
                                                           const bf16* __restrict__ dO, long lddo,
                                                           const float* __restrict__ lse,
                                                           float* __restrict__ delta, bf16* __restrict__ dQ,
                                                           long lddq, float scale) {
  constexpr int NB = CMHAR_ATTN_DQ_NBUF;
  static_assert(NB == 2 || NB == 3, "two or three K/V buffers");
  __shared__ __attribute__((aligned(16))) char smem[NB * 16384];
#undef Ks
#undef Vs
#define Ks(buf) (smem + 8192 * (buf))
#define Vs(buf) (smem + 8192 * NB + 8192 * (buf))
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const BlkIdx bi = flash_block(H);
  const int hd = bi.hd, b = bi.b;
  const int q0 = q_base + bi.blk * (128 * QB) + wave * (32 * QB);
  const bf16* Kb = K + (long)b * Lk * ldk + hd * 64;
  const bf16* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * LOG2E;
  bf16x8 qf[QB][4], gf[QB][4];
  float sL[QB], Dl[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int myq = min(q0 + 32 * j + (lane & 31), Lq - 1);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      qf[j][t] = *(const bf16x8*)(Q + ((long)b * Lq + myq) * ldq + hd * 64 + 16 * t + 8 * h);
      gf[j][t] = *(const bf16x8*)(dO + ((long)b * Lq + myq) * lddo + hd * 64 + 16 * t + 8 * h);
    }
    sL[j] = -lse[((long)b * H + hd) * Lq + myq] / c;    // accumulator seed: p = exp2(c·acc)
    float d_ = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8 ov = *(const bf16x8*)(O + ((long)b * Lq + myq) * ldo + hd * 64 + 16 * t + 8 * h);
#pragma unroll
      for (int e = 0; e < 8; ++e) d_ = fmaf((float)gf[j][t][e], (float)ov[e], d_);
    }
    d_ = pair_sum(d_);
    Dl[j] = d_;
    if (h == 0 && q0 + 32 * j + (lane & 31) < Lq) delta[((long)b * H + hd) * Lq + myq] = d_;
  }
  // (register operands retired here, before the tile loop: otherwise the compiler's wait for these loads sits inside
  // the loop, counted as if its own loads were the only memory operations in flight — with the DMA issued by inline
  // asm (CMHAR_ATTN_ASM_DMA) that stalled every tile on the next tile's DMA)
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    asm volatile("" :: "v"(sL[j]), "v"(Dl[j]));
#pragma unroll
    for (int t = 0; t < 4; ++t) asm volatile("" :: "v"(qf[j][t]), "v"(gf[j][t]));
  }
  floatx16 dq[QB][2];
#pragma unroll
  for (int j = 0; j < QB; ++j)
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[j][d][r] = 0.f;
  const int nt = (Lk + 63) / 64;
  TileDma tk, tv;
  tk.init(Kb, ldk, Lk, wave, lane);
  tv.init(Vb, ldv, Lk, wave, lane);
  tk.tile(0, Ks(0), wave);
  tv.tile(0, Vs(0), wave);
  if (NB == 3 && nt > 1) {
    tk.tile(64, Ks(1), wave);
    tv.tile(64, Vs(1), wave);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const bool active = q0 < Lq;      // waves past the last query only stage tiles and join barriers (see forward)
  // one tile per call, LDS buffer index a compile-time constant (tiles run in pairs / triples): LDS addresses fold
  // into the ds_read immediate offsets
  auto tile = [&](auto CUR, int kt) __attribute__((always_inline)) {
    constexpr int cur = decltype(CUR)::value;
    const bool more = kt + 1 < nt;
    // NB = 2: the next tile into the other buffer; NB = 3: the tile after next into the buffer the previous tile
    // used (its last reader passed the previous tile's barrier)
    const int ahead = NB - 1;
    const bool issue = kt + ahead < nt && !(CMHAR_ATTN_ABL_NODMA & 2);
    constexpr int nb = (cur + NB - 1) % NB;
    constexpr int pos = CMHAR_ATTN_DMA_POS;
    if (issue && (pos != 1 || !active)) tk.tile((kt + ahead) * 64, Ks(nb), wave);
    if (issue && (pos == 0 || !active)) tv.tile((kt + ahead) * 64, Vs(nb), wave);
    const int kbase = kt * 64;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (!active) break;
      floatx16 s[QB], dp[QB];
#pragma unroll
      for (int j = 0; j < QB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[j][r] = sL[j]; dp[j][r] = -Dl[j]; }
      PRIO_HI();
#pragma unroll
      for (int t = 0; t < 4; ++t) {    // each K / V row fragment read once, used by all QB q-blocks
        const bf16x8 kfr = row_frag(Ks(cur), kb * 32, t, lane);
        const bf16x8 vfr = row_frag(Vs(cur), kb * 32, t, lane);
#pragma unroll
        for (int j = 0; j < QB; ++j) {
          s[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr, qf[j][t], s[j], 0, 0, 0);
          dp[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr, gf[j][t], dp[j], 0, 0, 0);
        }
      }
      PRIO_LO();
      if (pos != 0 && kb == 0 && issue) {
        __builtin_amdgcn_sched_barrier(0);
        if (pos == 1) tk.tile((kt + ahead) * 64, Ks(nb), wave);
        tv.tile((kt + ahead) * 64, Vs(nb), wave);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (kbase + 64 > Lk) {   // ragged last tile only (wave-uniform branch)
#pragma unroll
        for (int j = 0; j < QB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kbase + kb * 32 + acc_row(r, h) >= Lk) s[j][r] = -INFINITY;
      }
      bf16x8 db[QB][2];
#pragma unroll
      for (int j = 0; j < QB; ++j) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) {   // aligned pairs: one v_pk_mul_f32 + one v_cvt_pk_bf16_f32 each
          const float2_t pv = PS ? float2_t{fexp2(s[j][r]), fexp2(s[j][r + 1])}
                                 : float2_t{fexp2(s[j][r] * c), fexp2(s[j][r + 1] * c)};
          const bf16x2_t dd = __builtin_convertvector(pv * float2_t{dp[j][r], dp[j][r + 1]}, bf16x2_t);
          db[j][r >> 3][r & 7] = dd[0];
          db[j][r >> 3][(r & 7) + 1] = dd[1];
        }
      }
      PRIO_HI();
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const bf16x8 ktr = tr_frag(Ks(cur), kb * 32, ss, d * 32, lane);
#pragma unroll
          for (int j = 0; j < QB; ++j)
            dq[j][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ktr, db[j][ss], dq[j][d], 0, 0, 0);
        }
      PRIO_LO();
    }
    if (more) {   // own pieces of the next tile landed (NB = 3: the tile after it still in flight)
      if (issue && NB == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };
  if constexpr (NB == 3) {
    for (int kt = 0; kt < nt; kt += 3) {
      tile(std::integral_constant<int, 0>{}, kt);
      if (kt + 1 < nt) tile(std::integral_constant<int, 1>{}, kt + 1);
      if (kt + 2 < nt) tile(std::integral_constant<int, 2>{}, kt + 2);
    }
  } else {
    for (int kt = 0; kt < nt; kt += 2) {
      tile(std::integral_constant<int, 0>{}, kt);
      if (kt + 1 < nt) tile(std::integral_constant<int, 1>{}, kt + 1);
    }
  }
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int q = q0 + 32 * j + (lane & 31);
    if (q < Lq) store_row64<bf16>(dQ + ((long)b * Lq + q) * lddq + hd * 64, dq[j], scale, h);
  }
}
#undef Ks
#undef Vs

template <typename E>
__global__ __launch_bounds__(256, 2) void attn_fwd_tail_bf16(int H, int Lq, int Lk, int q_base0,
                                                             const bf16* __restrict__ Q, long ldq,
                                                             const bf16* __restrict__ K, long ldk,
                                                             const bf16* __restrict__ V, long ldv, E* __restrict__ O,
                                                             long ldo, float* __restrict__ lse, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[65536];   // grid.x = ⌈tail / 32⌉ groups of 32 rows
  fwd_tail_group<E, 2>(smem, H, Lq, Lk, q_base0 + 32 * blockIdx.x, blockIdx.y, blockIdx.z, Q, ldq, K, ldk, V, ldv, O,
                       ldo, lse, scale);
}
template <bool PS>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_tail_bf16(int H, int Lq, int Lk, int q_base0,
                                                                const bf16* __restrict__ Q, long ldq,
                                                                const bf16* __restrict__ K, long ldk,
                                                                const bf16* __restrict__ V, long ldv,
                                                                const bf16* __restrict__ O, long ldo,
                                                                const bf16* __restrict__ dO, long lddo,
                                                                const float* __restrict__ lse,
                                                                float* __restrict__ delta, bf16* __restrict__ dQ,
                                                                long lddq, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[65536];   // [2 buf][K 16 KB | V 16 KB]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const int hd = blockIdx.y, b = blockIdx.z;
  const int q_base = q_base0 + 32 * blockIdx.x;   // grid.x = ⌈tail / 32⌉ groups of 32 rows
  const bf16* Kb = K + (long)b * Lk * ldk + hd * 64;
  const bf16* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * LOG2E;
  const int myq = min(q_base + (lane & 31), Lq - 1);
  bf16x8 qf[4], gf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    qf[t] = *(const bf16x8*)(Q + ((long)b * Lq + myq) * ldq + hd * 64 + 16 * t + 8 * h);
    gf[t] = *(const bf16x8*)(dO + ((long)b * Lq + myq) * lddo + hd * 64 + 16 * t + 8 * h);
  }
  const float sL = -lse[((long)b * H + hd) * Lq + myq] / c;
  float Dl = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x8 ov = *(const bf16x8*)(O + ((long)b * Lq + myq) * ldo + hd * 64 + 16 * t + 8 * h);
#pragma unroll
    for (int e = 0; e < 8; ++e) Dl = fmaf((float)gf[t][e], (float)ov[e], Dl);
  }
  Dl += xhalf(Dl);
  if (wave == 0 && h == 0 && q_base + (lane & 31) < Lq) delta[((long)b * H + hd) * Lq + myq] = Dl;
  floatx16 dq[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
  const int nt = (Lk + 127) / 128;
  TileDma tk, tv;
  tk.init(Kb, ldk, Lk, wave, lane);
  tv.init(Vb, ldv, Lk, wave, lane);
  stage128(tk, 0, smem, wave);
  stage128(tv, 0, smem + 16384, wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int sub = (wave >> 1) * 8192, r0 = 32 * (wave & 1);
  for (int st = 0; st < nt; ++st) {
    char* Ks_ = smem + (st & 1) * 32768;
    char* Vs_ = Ks_ + 16384;
    const bool more = st + 1 < nt;
    if (more) {
      stage128(tk, (st + 1) * 128, smem + ((st + 1) & 1) * 32768, wave);
      stage128(tv, (st + 1) * 128, smem + ((st + 1) & 1) * 32768 + 16384, wave);
    }
    const int kbase = st * 128 + 32 * wave;
    if (kbase < Lk) {
      floatx16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = sL; dp[r] = -Dl; }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Ks_ + sub, r0, t, lane), qf[t], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Vs_ + sub, r0, t, lane), gf[t], dp, 0, 0, 0);
      }
      if (kbase + 32 > Lk) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + acc_row(r, h) >= Lk) s[r] = -INFINITY;
      }
      bf16x8 db[2];
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float2_t pv = PS ? float2_t{fexp2(s[r]), fexp2(s[r + 1])} : float2_t{fexp2(s[r] * c), fexp2(s[r + 1] * c)};
        const bf16x2_t dd = __builtin_convertvector(pv * float2_t{dp[r], dp[r + 1]}, bf16x2_t);
        db[r >> 3][r & 7] = dd[0];
        db[r >> 3][(r & 7) + 1] = dd[1];
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < 2; ++d)
          dq[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Ks_ + sub, r0, ss, d * 32, lane), db[ss], dq[d], 0, 0,
                                                          0);
    }
    if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float* Dw = (float*)smem;            // [4][32][64]
  const int ql = lane & 31;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) Dw[(wave * 32 + ql) * 64 + d * 32 + acc_row(r, h)] = dq[d][r];
  __syncthreads();
  const int qi = tid >> 3, d0 = (tid & 7) * 8;
  const int q = q_base + qi;
  if (q < Lq) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) a += Dw[(w * 32 + qi) * 64 + d0 + j];
      v[j] = (bf16)(a * scale);
    }
    *(bf16x8*)(dQ + ((long)b * Lq + q) * lddq + hd * 64 + d0) = v;
  }
}

template <bool PS>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_tail_bf16(int H, int Lq, int Lk, int k_base0,
                                                                  const bf16* __restrict__ Q, long ldq,
                                                                  const bf16* __restrict__ K, long ldk,
                                                                  const bf16* __restrict__ V, long ldv,
                                                                  const bf16* __restrict__ dO, long lddo,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ delta,
                                                                  bf16* __restrict__ dK, long lddk,
                                                                  bf16* __restrict__ dV, long lddv, float scale,
                                                                  float kscale) {
  __shared__ __attribute__((aligned(16))) char smem[65536 + 2 * 2 * 128 * 4];   // grid.x = ⌈tail / 32⌉ key groups
  dkdv_tail_group<PS, 2>(smem, H, Lq, Lk, k_base0 + 32 * blockIdx.x, blockIdx.y, blockIdx.z, Q, ldq, K, ldk, V, ldv, dO,
                         lddo, lse, delta, dK, lddk, dV, lddv, scale, kscale);
}

// ---------------------------------------------------------------------------------------------------------------
// exact fp32 path (any head dim <= 64), with optional attention-prob dropout (nn.MultiheadAttention semantics)
// ---------------------------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(64) void attn_fwd_f32(int H, int Lq, int Lk, const T* __restrict__ Q, long ldq, const T* __restrict__ K,
                             long ldk, const T* __restrict__ V, long ldv, T* __restrict__ O, long ldo,
                             float* __restrict__ lse, float scale, float pdrop, unsigned long long seed) {
  const int hd = blockIdx.y, b = blockIdx.z;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ float sK[64][D], sV[64][D];
  float qv[D], o[D];
  const bool active = q < Lq;
  const int qq = active ? q : 0;
#pragma unroll
  for (int d = 0; d < D; ++d) { qv[d] = to_f<T>(Q[((long)b * Lq + qq) * ldq + hd * D + d]) * scale; o[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const unsigned bh = b * H + hd;
  for (int k0 = 0; k0 < Lk; k0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * D; i += blockDim.x) {
      const int kk = i / D, d = i % D;
      const bool ok = k0 + kk < Lk;
      sK[kk][d] = ok ? to_f<T>(K[((long)b * Lk + k0 + kk) * ldk + hd * D + d]) : 0.f;
      sV[kk][d] = ok ? to_f<T>(V[((long)b * Lk + k0 + kk) * ldv + hd * D + d]) : 0.f;
    }
    __syncthreads();
    attn_row_f32<D>(qv, o, m, l, &sK[0][0], D, &sV[0][0], D, min(64, Lk - k0), seed, pdrop, bh, qq, k0);
  }
  if (active) {
#pragma unroll
    for (int d = 0; d < D; ++d) O[((long)b * Lq + q) * ldo + hd * D + d] = from_f<T>(o[d] / l);
    lse[((long)bh) * Lq + q] = m + __logf(l);     // natural-log LSE of scale*s
  }
}

template <typename T, int D>
__global__ __launch_bounds__(64) void attn_bwd_dq_f32(int H, int Lq, int Lk, const T* __restrict__ Q, long ldq, const T* __restrict__ K,
                                long ldk, const T* __restrict__ V, long ldv, const T* __restrict__ O, long ldo,
                                const T* __restrict__ dO, long lddo, const float* __restrict__ lse,
                                float* __restrict__ delta_out, T* __restrict__ dQ, long lddq, float scale,
                                float pdrop, unsigned long long seed) {
  const int hd = blockIdx.y, b = blockIdx.z;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ float sK[64][D], sV[64][D];
  const bool active = q < Lq;
  const int qq = active ? q : 0;
  const unsigned bh = b * H + hd;
  float qv[D], g[D], dq[D];
  float delta = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    qv[d] = to_f<T>(Q[((long)b * Lq + qq) * ldq + hd * D + d]) * scale;
    g[d] = to_f<T>(dO[((long)b * Lq + qq) * lddo + hd * D + d]);
    delta = fmaf(g[d], to_f<T>(O[((long)b * Lq + qq) * ldo + hd * D + d]), delta);   // explicit: as the fused IMU kernel
    dq[d] = 0.f;
  }
  const float L = lse[(long)bh * Lq + qq];
  for (int k0 = 0; k0 < Lk; k0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * D; i += blockDim.x) {
      const int kk = i / D, d = i % D;
      const bool ok = k0 + kk < Lk;
      sK[kk][d] = ok ? to_f<T>(K[((long)b * Lk + k0 + kk) * ldk + hd * D + d]) : 0.f;
      sV[kk][d] = ok ? to_f<T>(V[((long)b * Lk + k0 + kk) * ldv + hd * D + d]) : 0.f;
    }
    __syncthreads();
    attn_row_dq_f32<D>(qv, g, L, delta, dq, &sK[0][0], D, &sV[0][0], D, min(64, Lk - k0), seed, pdrop, bh, qq, k0);
  }
  if (active) {
#pragma unroll
    for (int d = 0; d < D; ++d) dQ[((long)b * Lq + q) * lddq + hd * D + d] = from_f<T>(dq[d] * scale);
    delta_out[(long)bh * Lq + q] = delta;
  }
}

template <typename T, int D>
__global__ __launch_bounds__(64) void attn_bwd_dkdv_f32(int H, int Lq, int Lk, const T* __restrict__ Q, long ldq,
                                  const T* __restrict__ K, long ldk, const T* __restrict__ V, long ldv,
                                  const T* __restrict__ dO, long lddo, const float* __restrict__ lse,
                                  const float* __restrict__ delta, T* __restrict__ dK, long lddk,
                                  T* __restrict__ dV, long lddv, float scale, float pdrop,
                                  unsigned long long seed) {
  const int hd = blockIdx.y, b = blockIdx.z;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ float sQ[64][D], sG[64][D], Ls[64], Ds[64];
  const bool active = k < Lk;
  const int kk = active ? k : 0;
  const unsigned bh = b * H + hd;
  float kv[D], vv[D], dk[D], dv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    kv[d] = to_f<T>(K[((long)b * Lk + kk) * ldk + hd * D + d]);
    vv[d] = to_f<T>(V[((long)b * Lk + kk) * ldv + hd * D + d]);
    dk[d] = 0.f;
    dv[d] = 0.f;
  }
  for (int q0 = 0; q0 < Lq; q0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * D; i += blockDim.x) {
      const int qi = i / D, d = i % D;
      const bool ok = q0 + qi < Lq;
      sQ[qi][d] = ok ? to_f<T>(Q[((long)b * Lq + q0 + qi) * ldq + hd * D + d]) * scale : 0.f;
      sG[qi][d] = ok ? to_f<T>(dO[((long)b * Lq + q0 + qi) * lddo + hd * D + d]) : 0.f;
    }
    for (int i = threadIdx.x; i < 64; i += blockDim.x) {
      const bool ok = q0 + i < Lq;
      Ls[i] = ok ? lse[(long)bh * Lq + q0 + i] : 0.f;
      Ds[i] = ok ? delta[(long)bh * Lq + q0 + i] : 0.f;
    }
    __syncthreads();
    // sQ already carries the scale (qs = 1)
    attn_row_dkdv_f32<D>(kv, vv, dk, dv, &sQ[0][0], D, 1.f, &sG[0][0], D, Ls, Ds, min(64, Lq - q0), seed, pdrop, bh,
                         q0, kk);
  }
  if (active) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      dK[((long)b * Lk + k) * lddk + hd * D + d] = from_f<T>(dk[d]);
      dV[((long)b * Lk + k) * lddv + hd * D + d] = from_f<T>(dv[d]);
    }
  }
}

#undef Ks
#undef Vs
#undef Qs
#undef Gs
}  // namespace

// QB = 2 for the dQ kernel does not fit 256 registers (spills at occupancy 2; at occupancy 1 it measured 16 % slower
// than QB = 1): off unless CMHAR_ATTN_DQ_QB=2 at build time (A/B builds only)
#ifndef CMHAR_ATTN_DQ_QB
#define CMHAR_ATTN_DQ_QB 1
#endif
// the ragged-tail kernels take tails of up to this many rows, in workgroups of 32 (0: off, the partly active blocks
// run them; A/B knob).  64: the 32-frame geometry's L = 3136 = 12·256 + 64 (forward) = 24·128 + 64 (dK/dV) tails.
#ifndef CMHAR_ATTN_TAIL
#define CMHAR_ATTN_TAIL 64
#endif
// 1: the tail groups run inside the bulk launch (first dispatched; see fwd_tail_group); 0: a tail launch of their own
// after the bulk.  Measured in one process at B = 32, H = 12, L = 1568 (tools/debug/attn_ab.py, µs per layer, two
// sessions): dK/dV folded 892.8 / 888.1 → 883.6 / 882.3 (backward), kept; the forward folded 339.8 → 323.5
// (round 6, after the round-5 A/B was found to launch the QB=1 kernel over the folded rows a second time), output
// bit-identical to the stand-alone tail kernel (tools/debug/attn_rowdiff.py) — kept (A/B knobs)
#ifndef CMHAR_ATTN_FOLD
#define CMHAR_ATTN_FOLD 1
#endif
#ifndef CMHAR_ATTN_FOLD_FWD
#define CMHAR_ATTN_FOLD_FWD 1
#endif

// f32-MFMA flash kernels (csrc/attention_f32.hip) for fp32 storage, D = 64, no dropout
void cmhar_attn_f32m_fwd(int B, int H, int Lq, int Lk, const float* Q, long ldq, const float* K, long ldk,
                         const float* V, long ldv, float* O, long ldo, float* lse, float scale, hipStream_t st);
void cmhar_attn_f32m_bwd(int B, int H, int Lq, int Lk, const float* Q, long ldq, const float* K, long ldk,
                         const float* V, long ldv, const float* O, long ldo, const float* dO, long lddo,
                         const float* lse, float* delta, float* dQ, long lddq, float* dK, long lddk, float* dV,
                         long lddv, float scale, hipStream_t st);

// every operand a 16-B aligned base with a row stride of whole 16-B chunks (the f32 flash tiles load float4s)
static bool f32m_ok(int dtype, int D, float pdrop, std::initializer_list<std::pair<const void*, long>> ops) {
  if (dtype != CMHAR_F32 || D != 64 || pdrop != 0.f || !cmhar_f32_mfma()) return false;
  for (const auto& o : ops)
    if (((uintptr_t)o.first & 15) || (o.second & 3)) return false;
  return true;
}

// The optimistic forward's workgroup flags: one zeroed int block per (device, stream), grown (never freed: a launch
// still in flight may hold the old one) to the largest bulk grid seen; every flag is 0 again after each forward
// (set by the optimistic launch, cleared by the gated exact launch behind it on the same stream).
static int* fwd_flags(hipStream_t st, long n) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<int*, long>> blocks;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto& e = blocks[{dev, st}];
  if (e.first && e.second >= n) return e.first;
  void* p = nullptr;
  if (hipMalloc(&p, n * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, n * sizeof(int), st) != hipSuccess) return nullptr;
  e = {(int*)p, n};
  return (int*)p;
}
static std::atomic<int> g_fwd_opt{-1};   // -1: CMHAR_ATTN_FWD_OPT from the environment (default: the build's)
static bool fwd_opt_on() {
  int v = g_fwd_opt.load();
  if (v < 0) {
    const char* s = getenv("CMHAR_ATTN_FWD_OPT");
    v = s ? (atoi(s) != 0) : (CMHAR_ATTN_FWD_OPT != 0);
    g_fwd_opt.store(v);
  }
  return v != 0;
}

// ----------------------------------------------------------------------------------------------------------------
// C ABI.  Tensors are [B*L, ld] row-major with head h at columns h*D .. h*D+D-1.
// lse / delta: fp32 [B*H*Lq] workspaces owned by the caller.
// ----------------------------------------------------------------------------------------------------------------
// The bf16 / fp16 flash forward's bulk launch: optimistic + gated exact (1) or one exact launch (0); mode < 0 only
// queries.  Returns the previous mode.
extern "C" int cmhar_attention_fwd_opt(int mode) {
  const int prev = fwd_opt_on() ? 1 : 0;
  if (mode >= 0) g_fwd_opt.store(mode != 0);
  return prev;
}
extern "C" int cmhar_attention_fwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* Q, long ldq,
                                   const void* K, long ldk, const void* V, long ldv, void* O, long ldo, float* lse,
                                   float scale, float pdrop, unsigned long long seed, hipStream_t st) {
  if (B <= 0 || Lq <= 0) return 0;
  if ((dtype == CMHAR_BF16 || dtype == CMHAR_F16) && D == 64 && pdrop == 0.f) {
    // 256-query workgroups (64 rows per wave) over the bulk, 128-query workgroups (32 rows per wave, waves past Lq
    // skip the math) for the rest
    // (CMHAR_ATTN_FWD_ONE_LAUNCH: 256-query workgroups everywhere, the last one per head partly idle)
    const int bulk = CMHAR_ATTN_FWD_ONE_LAUNCH ? cdiv(Lq, 256) * 256 : (Lq / 256) * 256;
    const bool tail = Lq > bulk && Lq - bulk <= CMHAR_ATTN_TAIL;
    // the tail's 32-query groups folded into the bulk launch (tail_block), or a launch of their own
    const int fold = tail && bulk > 0 && CMHAR_ATTN_FOLD_FWD ? cdiv(Lq - bulk, 32) : 0;
    // the optimistic bulk launch and its gated exact rerun (see attn_fwd_bf16's OPT)
    int* const flags = bulk > 0 && fwd_opt_on() ? fwd_flags(st, (long)(bulk / 256 + fold) * H * B) : nullptr;
#define FL(E)                                                                                                    \
  do {                                                                                                           \
    if (bulk > 0 && flags) {                                                                                     \
      attn_fwd_bf16<E, 2, true><<<dim3(bulk / 256 + fold, H, B), 256, 0, st>>>(                                  \
          H, Lq, Lk, 0, (const bf16*)Q, ldq, (const bf16*)K, ldk, (const bf16*)V, ldv, (E*)O, ldo, lse, scale, fold, \
          bulk, flags);                                                                                          \
      attn_fwd_bf16<E, 2><<<dim3(bulk / 256 + fold, H, B), 256, 0, st>>>(H, Lq, Lk, 0, (const bf16*)Q, ldq,         \
                                                                         (const bf16*)K, ldk, (const bf16*)V, ldv, \
                                                                         (E*)O, ldo, lse, scale, fold, bulk,     \
                                                                         flags);                                 \
    } else if (bulk > 0)                                                                                         \
      attn_fwd_bf16<E, 2><<<dim3(bulk / 256 + fold, H, B), 256, 0, st>>>(H, Lq, Lk, 0, (const bf16*)Q, ldq,         \
                                                                         (const bf16*)K, ldk, (const bf16*)V, ldv, \
                                                                         (E*)O, ldo, lse, scale, fold, bulk,     \
                                                                         nullptr);                               \
    if (tail && !fold)                                                                                           \
      attn_fwd_tail_bf16<E><<<dim3(cdiv(Lq - bulk, 32), H, B), 256, 0, st>>>(H, Lq, Lk, bulk, (const bf16*)Q, ldq,   \
                                                                             (const bf16*)K, ldk,                \
                                                           (const bf16*)V, ldv, (E*)O, ldo, lse, scale);        \
    else if (Lq > bulk && !tail)   /* (folded tail groups: nothing left to launch) */                        \
      attn_fwd_bf16<E, 1><<<dim3(cdiv(Lq - bulk, 128), H, B), 256, 0, st>>>(H, Lq, Lk, bulk, (const bf16*)Q, ldq,   \
                                                                            (const bf16*)K, ldk, (const bf16*)V, ldv, \
                                                                            (E*)O, ldo, lse, scale, 0, 0, nullptr); \
  } while (0)
    if (dtype == CMHAR_F16) FL(f16); else FL(bf16);
#undef FL
  } else if (f32m_ok(dtype, D, pdrop, {{Q, ldq}, {K, ldk}, {V, ldv}, {O, ldo}})) {
    cmhar_attn_f32m_fwd(B, H, Lq, Lk, (const float*)Q, ldq, (const float*)K, ldk, (const float*)V, ldv, (float*)O, ldo,
                        lse, scale, st);
  } else {
    // exact-fp32 math path (fp32 storage, or bf16 storage with a head dim / dropout the flash kernel lacks);
    // its LSE is in natural-log units and is only ever consumed by the matching backward below
    dim3 grid(cdiv(Lq, 64), H, B);
#define F(TT, DD)                                                                                         \
  attn_fwd_f32<TT, DD><<<grid, 64, 0, st>>>(H, Lq, Lk, (const TT*)Q, ldq, (const TT*)K, ldk, (const TT*)V, ldv, \
                                            (TT*)O, ldo, lse, scale, pdrop, seed)
#define SW(TT) switch (D) { case 8: F(TT, 8); break; case 16: F(TT, 16); break; case 32: F(TT, 32); break;  \
                            case 64: F(TT, 64); break; default: return -1; }
    if (dtype == CMHAR_BF16) { SW(bf16) } else if (dtype == CMHAR_F16) { SW(f16) } else { SW(float) }
#undef SW
#undef F
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Backward.  delta: fp32 [B*H*Lq] workspace (written here).
// bf16 flash backward; PS: pre-scaled keys (see attn_bwd_dkdv_bf16), `scale` then the true softmax scale
template <bool PS>
static void flash_bwd_bf16(int B, int H, int Lq, int Lk, const void* Q, long ldq, const void* K, long ldk,
                           const void* V, long ldv, const void* O, long ldo, const void* dO, long lddo,
                           const float* lse, float* delta, void* dQ, long lddq, void* dK, long lddk, void* dV,
                           long lddv, float scale, hipStream_t st) {
  const float s_in = PS ? 1.f / LOG2E : scale;   // c = s_in·log2e (1 when PS) and the dQ output factor
  // 256-query workgroups (QB = 2) over the bulk, 128-query workgroups for the rest (as the forward)
  const int bulk = CMHAR_ATTN_DQ_QB == 2 ? (Lq / 256) * 256 : 0;
  if (bulk > 0)
    attn_bwd_dq_bf16<2, PS><<<dim3(bulk / 256, H, B), 256, 0, st>>>(H, Lq, Lk, 0, (const bf16*)Q, ldq, (const bf16*)K,
                                                                    ldk, (const bf16*)V, ldv, (const bf16*)O, ldo,
                                                                    (const bf16*)dO, lddo, lse, delta, (bf16*)dQ,
                                                                    lddq, s_in);
  // a tail of <= CMHAR_ATTN_TAIL queries / keys beyond the last full 128-row block goes to the tail kernels
  // (the dQ tail kernel measured slower than the in-grid one-active-wave block at L = 1568 — 351.6 + 31.8 µs vs 367.1
  // µs per layer — so it only takes sequences that are ALL tail, Lq <= CMHAR_ATTN_TAIL: the one-query rows of the
  // token-0 last layer, the cross-attention fusion's IMU queries)
  const int qfull = bulk + ((Lq - bulk) / 128) * 128;
  const bool qtail = qfull == 0 && Lq - qfull <= CMHAR_ATTN_TAIL;
  const int qend = qtail ? qfull : Lq;
  if (qend > bulk)
    attn_bwd_dq_bf16<1, PS><<<dim3(cdiv(qend - bulk, 128), H, B), 256, 0, st>>>(
        H, Lq, Lk, bulk, (const bf16*)Q, ldq, (const bf16*)K, ldk, (const bf16*)V, ldv, (const bf16*)O, ldo,
        (const bf16*)dO, lddo, lse, delta, (bf16*)dQ, lddq, s_in);
  if (qtail)
    attn_bwd_dq_tail_bf16<PS><<<dim3(cdiv(Lq - qfull, 32), H, B), 256, 0, st>>>(H, Lq, Lk, qfull, (const bf16*)Q, ldq,
                                                                                (const bf16*)K,
                                                             ldk, (const bf16*)V, ldv, (const bf16*)O, ldo,
                                                             (const bf16*)dO, lddo, lse, delta, (bf16*)dQ, lddq, s_in);
  const int kfull = (Lk / 128) * 128;
  const bool ktail = Lk > kfull && Lk - kfull <= CMHAR_ATTN_TAIL;
  const int kblocks = (ktail ? kfull : cdiv(Lk, 128) * 128) / 128;
  const int fold = ktail && kblocks > 0 && CMHAR_ATTN_FOLD ? cdiv(Lk - kfull, 32) : 0;   // as the forward
  if (kblocks > 0)
    attn_bwd_dkdv_bf16<PS><<<dim3(kblocks + fold, H, B), 256, 0, st>>>(H, Lq, Lk, 0, (const bf16*)Q, ldq,
                                                                       (const bf16*)K, ldk, (const bf16*)V, ldv,
                                                                       (const bf16*)dO, lddo, lse, delta, (bf16*)dK,
                                                                       lddk, (bf16*)dV, lddv, s_in, scale, fold, kfull);
  if (ktail && !fold)
    attn_bwd_dkdv_tail_bf16<PS><<<dim3(cdiv(Lk - kfull, 32), H, B), 256, 0, st>>>(H, Lq, Lk, kfull, (const bf16*)Q,
                                                                                  ldq, (const bf16*)K,
                                                               ldk, (const bf16*)V, ldv, (const bf16*)dO, lddo, lse,
                                                               delta, (bf16*)dK, lddk, (bf16*)dV, lddv, s_in, scale);
}

extern "C" int cmhar_attention_bwd_prescaled(int B, int H, int Lq, int Lk, const void* Q, long ldq, const void* K,
                                             long ldk, const void* V, long ldv, const void* O, long ldo,
                                             const void* dO, long lddo, const float* lse, float* delta, void* dQ,
                                             long lddq, void* dK, long lddk, void* dV, long lddv, float scale,
                                             hipStream_t st) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || !Q || !K || !V || !O || !dO || !lse || !delta || !dQ || !dK || !dV) return -1;
  flash_bwd_bf16<true>(B, H, Lq, Lk, Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, delta, dQ, lddq, dK, lddk, dV, lddv,
                       scale, st);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_attention_bwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* Q, long ldq,
                                   const void* K, long ldk, const void* V, long ldv, const void* O, long ldo,
                                   const void* dO, long lddo, const float* lse, float* delta, void* dQ, long lddq,
                                   void* dK, long lddk, void* dV, long lddv, float scale, float pdrop,
                                   unsigned long long seed, hipStream_t st) {
  if (B <= 0 || Lq <= 0) return 0;
  if (dtype == CMHAR_F16) return -1;   // fp16 is the inference-only path
  if (dtype == CMHAR_BF16 && D == 64 && pdrop == 0.f) {
    flash_bwd_bf16<false>(B, H, Lq, Lk, Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, delta, dQ, lddq, dK, lddk, dV,
                          lddv, scale, st);
  } else if (f32m_ok(dtype, D, pdrop, {{Q, ldq}, {K, ldk}, {V, ldv}, {O, ldo}, {dO, lddo}, {dQ, lddq}, {dK, lddk},
                                       {dV, lddv}})) {
    cmhar_attn_f32m_bwd(B, H, Lq, Lk, (const float*)Q, ldq, (const float*)K, ldk, (const float*)V, ldv,
                        (const float*)O, ldo, (const float*)dO, lddo, lse, delta, (float*)dQ, lddq, (float*)dK, lddk,
                        (float*)dV, lddv, scale, st);
  } else {
#define F(TT, DD)                                                                                               \
  attn_bwd_dq_f32<TT, DD><<<dim3(cdiv(Lq, 64), H, B), 64, 0, st>>>(H, Lq, Lk, (const TT*)Q, ldq, (const TT*)K, ldk,   \
                                                                   (const TT*)V, ldv, (const TT*)O, ldo,             \
                                                                   (const TT*)dO, lddo, lse, delta, (TT*)dQ, lddq,   \
                                                                   scale, pdrop, seed);                              \
  attn_bwd_dkdv_f32<TT, DD><<<dim3(cdiv(Lk, 64), H, B), 64, 0, st>>>(H, Lq, Lk, (const TT*)Q, ldq, (const TT*)K,      \
                                                                     ldk, (const TT*)V, ldv, (const TT*)dO, lddo,     \
                                                                     lse, delta, (TT*)dK, lddk, (TT*)dV, lddv, scale, \
                                                                     pdrop, seed)
#define SW(TT) switch (D) { case 8: F(TT, 8); break; case 16: F(TT, 16); break; case 32: F(TT, 32); break;  \
                            case 64: F(TT, 64); break; default: return -1; }
    if (dtype == CMHAR_BF16) { SW(bf16) } else { SW(float) }
#undef SW
#undef F
  }
  CMHAR_CHECK_LAUNCH();
  return 0;
}
