// Flash attention on the f32-input MFMA (v_mfma_f32_32x32x2_f32: f32 operands, f32 accumulate, exact f32 products)
// for the exact-fp32 parity mode's VideoMAE attention: head dim 64, fp32 storage, no dropout
// (third-party transformers modeling_videomae.py:209-258, softmax(QKᵀ/√d)V).  The algorithm is the bf16 flash path's
// (csrc/attention.hip) with f32 fragments: one f32 per lane per MFMA operand (lane l: A[i = l&31][k = l>>5],
// B[k = l>>5][j = l&31]), so a 64-wide head-dim contraction is 32 MFMAs of k = 2.
//   fwd   wave = 32 queries; Sᵀ = K·Qᵀ puts the query on the lane (Q·scale·log2e held in 32 registers), the online
//         softmax is lane-local (+1 cross-half exchange), and Pᵀ's accumulator registers ARE the B operand of
//         Oᵀ += Vᵀ·Pᵀ: accumulator register p of lane half h holds key (p&3) + 8(p>>2) + 4h, which is the k slot the
//         MFMA chain reads from that lane — no data movement between the two products.
//   dQ    wave = 32 queries (Q, dO in registers), Sᵀ and dPᵀ recomputed per 32-key block, dQᵀ += Kᵀ·dSᵀ; also
//         writes δ = rowsum(dO∘O) for the dK/dV kernel.
//   dK/dV wave = 32 keys (K, V in registers), S and dP with the key on the lane, their accumulators pre-loaded with
//         −lse·log2e and −δ of each query row, dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS.
// K/V (fwd, dQ) and Q/dO (dK/dV) stream through LDS as [64][64] f32 tiles, register-staged and double-buffered
// (loads for tile t+1 in flight under tile t's MFMAs), with a bit-level XOR swizzle that keeps both access patterns
// bank-conflict free: column reads (lane = row r, element 2p + h) and row reads (lane = element, row per lane half).
// LSE is in natural-log units, as the exact-f32 VALU kernels' (the pair is interchangeable per call).
#include "common.h"

namespace {

constexpr float F_LOG2E = 1.4426950408889634f;
constexpr float F_LN2 = 0.69314718055994531f;
constexpr int FTILE = 64 * 64;   // floats per LDS tile

__device__ __forceinline__ float f_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Row swizzle: bits 1..5 of the element index are XORed with a bijection of the row's low 5 bits, chosen so that
//   column reads  (32 lanes = 32 consecutive rows, elements d and d+1 in the two lane halves) hit 64 distinct banks
//     (rows differ in the bits 1..5 pattern; d and d+1 differ in bit 0), and
//   row reads     (32 lanes = 32 consecutive elements; the halves read rows ρ and ρ+4, which differ in row bit 2 →
//     element bit 5) hit disjoint 32-bank halves.
__device__ __forceinline__ int fsw(int r) { return ((r & 3) << 1) | (((r >> 3) & 3) << 3) | (((r >> 2) & 1) << 5); }
__device__ __forceinline__ int foff(int r, int d) { return r * 64 + (d ^ fsw(r)); }

// accumulator register q of lane half h ↔ row (q&3) + 8(q>>2) + 4h of a 32x32 block
__device__ __forceinline__ int frow(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

__device__ __forceinline__ float fxhalf(float v) { return __shfl_xor(v, 32); }

__device__ __forceinline__ floatx16 fmma(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// A 64-row x 64-float tile of a head slice (rows r0.., row stride ld), register-staged in two halves of 32 rows
// (2 float4 per thread, 16 threads per 256-B row, coalesced) so that only one half's 8 VGPRs per operand are live
// across the MFMA blocks; rows at or past `rows` read as zero; `mul` scales on the way into LDS.
struct FTileStage {
  floatx4 v[2];
  __device__ __forceinline__ void load(const float* __restrict__ P, long ld, int r0, int rows, int half, int tid) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = (2 * half + it) * 256 + tid, r = i >> 4, c = i & 15;
      v[it] = r0 + r < rows ? *(const floatx4*)(P + (long)(r0 + r) * ld + 4 * c) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ S, int half, int tid, float mul) const {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = (2 * half + it) * 256 + tid, r = i >> 4, c = i & 15, sw = fsw(r);
      floatx4 x = v[it] * mul;
      if (sw & 2) x = floatx4{x[2], x[3], x[0], x[1]};   // element bit 1 of the swizzle, inside the 16-B chunk
      *(floatx4*)(S + r * 64 + ((4 * c) ^ (sw & ~3))) = x;
    }
  }
  // whole tile at once (prologue)
  __device__ __forceinline__ void fill(const float* __restrict__ P, long ld, int r0, int rows, float* __restrict__ S,
                                       int tid, float mul) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      load(P, ld, r0, rows, half, tid);
      store(S, half, tid, mul);
    }
  }
};

// Write a wave's two 32x32 accumulators (rows = head dim d, columns = the wave's 32 rows ρ) as rows ρ of a
// row-major [rows][64] output, times `mul`: transposed through this wave's 8.25 KB of LDS so that each store
// instruction writes one 256-B row.
__device__ __forceinline__ void f_store_rows(const floatx16 (&acc)[2], const float* mul_per_lane, float* lds, float* dst,
                                             long ld, int row0, int rows, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const float mul = *mul_per_lane;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int q = 0; q < 16; ++q) lds[r * 65 + 32 * c + frow(q, h)] = acc[c][q] * mul;
  __builtin_amdgcn_wave_barrier();   // wave-private region: LDS ops of one wave complete in order
#pragma unroll 4
  for (int it = 0; it < 32; ++it)
    if (row0 + it < rows) dst[(long)(row0 + it) * ld + lane] = lds[it * 65 + lane];
}

// ---------------------------------------------------------------------------------------------------------------
// forward: O = softmax(scale·QKᵀ)V, lse = natural-log row LSE of scale·QKᵀ
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_fwd_f32m(int H, int Lq, int Lk, const float* __restrict__ Q, long ldq,
                                                       const float* __restrict__ K, long ldk,
                                                       const float* __restrict__ V, long ldv, float* __restrict__ O,
                                                       long ldo, float* __restrict__ lse, float scale) {
  __shared__ __attribute__((aligned(16))) float smem[4 * FTILE];   // K0 K1 V0 V1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r = lane & 31;
  const BlkIdx bi = flash_block(H);
  const int hd = bi.hd, b = bi.b;
  const int q0 = bi.blk * 128 + wave * 32;
  const float* Qb = Q + (long)b * Lq * ldq + hd * 64;
  const float* Kb = K + (long)b * Lk * ldk + hd * 64;
  const float* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * F_LOG2E;
  float qf[32];
  {
    const float* qrow = Qb + (long)min(q0 + r, Lq - 1) * ldq + h;
#pragma unroll
    for (int p = 0; p < 32; ++p) qf[p] = qrow[2 * p] * c;
  }
  floatx16 o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int q = 0; q < 16; ++q) o[d][q] = 0.f;
  float m = -INFINITY, l = 0.f;
  const bool active = q0 < Lq;
  const int nt = (Lk + 63) / 64;
  FTileStage sk, sv;
  sk.fill(Kb, ldk, 0, Lk, smem, tid, 1.f);
  sv.fill(Vb, ldv, 0, Lk, smem + 2 * FTILE, tid, 1.f);
  __syncthreads();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nt;
    const float* Ks = smem + cur * FTILE;
    const float* Vs = smem + (2 + cur) * FTILE;
#pragma unroll 1
    for (int kb = 0; kb < 2; ++kb) {
      if (more) {   // half kb of the next K/V tile in flight under this block's MFMAs
        sk.load(Kb, ldk, (kt + 1) * 64, Lk, kb, tid);
        sv.load(Vb, ldv, (kt + 1) * 64, Lk, kb, tid);
      }
      if (active) {
        floatx16 s;
#pragma unroll
        for (int q = 0; q < 16; ++q) s[q] = 0.f;
#pragma unroll
        for (int p = 0; p < 32; ++p) s = fmma(Ks[foff(kb * 32 + r, 2 * p + h)], qf[p], s);
        const int kbase = kt * 64 + kb * 32;
        if (kbase + 32 > Lk) {   // ragged last block (wave-uniform)
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (kbase + frow(q, h) >= Lk) s[q] = -INFINITY;
        }
        float mt = s[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) mt = fmaxf(mt, s[q]);
        mt = fmaxf(mt, fxhalf(mt));
        const float mn = fmaxf(m, mt);   // finite: block 0 of tile 0 always holds key 0
        const float alpha = f_exp2(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int q = 0; q < 16; ++q) o[d][q] *= alpha;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          s[q] = f_exp2(s[q] - mn);
          l += s[q];
        }
#pragma unroll
        for (int p = 0; p < 16; ++p) {
          const int row = kb * 32 + frow(p, h);
          o[0] = fmma(Vs[foff(row, r)], s[p], o[0]);
          o[1] = fmma(Vs[foff(row, 32 + r)], s[p], o[1]);
        }
      }
      if (more) {
        sk.store(smem + (cur ^ 1) * FTILE, kb, tid, 1.f);
        sv.store(smem + (2 + (cur ^ 1)) * FTILE, kb, tid, 1.f);
      }
    }
    __syncthreads();
  }
  if (!active) return;
  l += fxhalf(l);
  const float inv = 1.f / l;
  f_store_rows(o, &inv, smem + wave * 2112, O + (long)b * Lq * ldo + hd * 64, ldo, q0, Lq, lane);
  if (h == 0 && q0 + r < Lq) lse[(long)(b * H + hd) * Lq + q0 + r] = (m + log2f(l)) * F_LN2;
}

// ---------------------------------------------------------------------------------------------------------------
// backward: dQ (and δ)
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_f32m(int H, int Lq, int Lk, const float* __restrict__ Q,
                                                          long ldq, const float* __restrict__ K, long ldk,
                                                          const float* __restrict__ V, long ldv,
                                                          const float* __restrict__ O, long ldo,
                                                          const float* __restrict__ dO, long lddo,
                                                          const float* __restrict__ lse, float* __restrict__ delta_out,
                                                          float* __restrict__ dQ, long lddq, float scale) {
  __shared__ __attribute__((aligned(16))) float smem[4 * FTILE];   // K0 K1 V0 V1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r = lane & 31;
  const BlkIdx bi = flash_block(H);
  const int hd = bi.hd, b = bi.b;
  const int q0 = bi.blk * 128 + wave * 32;
  const long bh = (long)b * H + hd;
  const float* Kb = K + (long)b * Lk * ldk + hd * 64;
  const float* Vb = V + (long)b * Lk * ldv + hd * 64;
  const float c = scale * F_LOG2E;
  const int myq = min(q0 + r, Lq - 1);
  float qf[32], gf[32];
  float delta = 0.f;
  {
    const long qo = (long)b * Lq + myq;
    const float* qrow = Q + qo * ldq + hd * 64 + h;
    const float* grow = dO + qo * lddo + hd * 64 + h;
    const float* orow = O + qo * ldo + hd * 64 + h;
#pragma unroll
    for (int p = 0; p < 32; ++p) {
      qf[p] = qrow[2 * p] * c;
      gf[p] = grow[2 * p];
      delta = fmaf(gf[p], orow[2 * p], delta);
    }
  }
  delta += fxhalf(delta);
  const float lse2 = lse[bh * Lq + myq] * F_LOG2E;
  floatx16 dq[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int q = 0; q < 16; ++q) dq[d][q] = 0.f;
  const bool active = q0 < Lq;
  const int nt = (Lk + 63) / 64;
  FTileStage sk, sv;
  sk.fill(Kb, ldk, 0, Lk, smem, tid, 1.f);
  sv.fill(Vb, ldv, 0, Lk, smem + 2 * FTILE, tid, 1.f);
  __syncthreads();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nt;
    const float* Ks = smem + cur * FTILE;
    const float* Vs = smem + (2 + cur) * FTILE;
#pragma unroll 1
    for (int kb = 0; kb < 2; ++kb) {
      if (more) {
        sk.load(Kb, ldk, (kt + 1) * 64, Lk, kb, tid);
        sv.load(Vb, ldv, (kt + 1) * 64, Lk, kb, tid);
      }
      if (active) {
        floatx16 s, dp;
#pragma unroll
        for (int q = 0; q < 16; ++q) { s[q] = 0.f; dp[q] = 0.f; }
#pragma unroll
        for (int p = 0; p < 32; ++p) {
          s = fmma(Ks[foff(kb * 32 + r, 2 * p + h)], qf[p], s);
          dp = fmma(Vs[foff(kb * 32 + r, 2 * p + h)], gf[p], dp);
        }
        const int kbase = kt * 64 + kb * 32;
        const bool ragged = kbase + 32 > Lk;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          float pr = f_exp2(s[q] - lse2);
          if (ragged && kbase + frow(q, h) >= Lk) pr = 0.f;
          s[q] = pr * (dp[q] - delta);   // dSᵀ
        }
#pragma unroll
        for (int p = 0; p < 16; ++p) {
          const int row = kb * 32 + frow(p, h);
          dq[0] = fmma(Ks[foff(row, r)], s[p], dq[0]);
          dq[1] = fmma(Ks[foff(row, 32 + r)], s[p], dq[1]);
        }
      }
      if (more) {
        sk.store(smem + (cur ^ 1) * FTILE, kb, tid, 1.f);
        sv.store(smem + (2 + (cur ^ 1)) * FTILE, kb, tid, 1.f);
      }
    }
    __syncthreads();
  }
  if (!active) return;
  f_store_rows(dq, &scale, smem + wave * 2112, dQ + (long)b * Lq * lddq + hd * 64, lddq, q0, Lq, lane);
  if (h == 0 && q0 + r < Lq) delta_out[bh * Lq + q0 + r] = delta;
}

// ---------------------------------------------------------------------------------------------------------------
// backward: dK, dV
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_f32m(int H, int Lq, int Lk, const float* __restrict__ Q,
                                                            long ldq, const float* __restrict__ K, long ldk,
                                                            const float* __restrict__ V, long ldv,
                                                            const float* __restrict__ dO, long lddo,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta, float* __restrict__ dK,
                                                            long lddk, float* __restrict__ dV, long lddv,
                                                            float scale) {
  __shared__ __attribute__((aligned(16))) float smem[4 * FTILE];   // Q0 Q1 G0 G1 (G = dO)
  __shared__ float rowc[2][2][64];                                  // [buf][−lse·log2e | −δ][query]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r = lane & 31;
  const BlkIdx bi = flash_block(H);
  const int hd = bi.hd, b = bi.b;
  const int k0 = bi.blk * 128 + wave * 32;
  const long bh = (long)b * H + hd;
  const float* Qb = Q + (long)b * Lq * ldq + hd * 64;
  const float* Gb = dO + (long)b * Lq * lddo + hd * 64;
  const float c = scale * F_LOG2E;
  float kf[32], vf[32];
  {
    const long ko = (long)b * Lk + min(k0 + r, Lk - 1);
    const float* krow = K + ko * ldk + hd * 64 + h;
    const float* vrow = V + ko * ldv + hd * 64 + h;
#pragma unroll
    for (int p = 0; p < 32; ++p) { kf[p] = krow[2 * p]; vf[p] = vrow[2 * p]; }
  }
  floatx16 dk[2], dv[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int q = 0; q < 16; ++q) { dk[d][q] = 0.f; dv[d][q] = 0.f; }
  const bool active = k0 < Lk;
  const int nt = (Lq + 63) / 64;
  // row constants of query tile t (threads 0..63: −lse·log2e, threads 64..127: −δ; padded queries: −∞ and 0, so
  // their P and dS are exactly 0)
  auto rowconst = [&](int t) -> float {
    const int i = tid & 63, q = t * 64 + i;
    if (tid < 64) return q < Lq ? -lse[bh * Lq + q] * F_LOG2E : -INFINITY;
    return q < Lq ? -delta[bh * Lq + q] : 0.f;
  };
  FTileStage sq, sg;
  float rc = 0.f;
  sq.fill(Qb, ldq, 0, Lq, smem, tid, c);
  sg.fill(Gb, lddo, 0, Lq, smem + 2 * FTILE, tid, 1.f);
  if (tid < 128) rowc[0][tid >> 6][tid & 63] = rowconst(0);
  __syncthreads();
  for (int qt = 0; qt < nt; ++qt) {
    const int cur = qt & 1;
    const bool more = qt + 1 < nt;
    if (more && tid < 128) rc = rowconst(qt + 1);
    const float* Qs = smem + cur * FTILE;
    const float* Gs = smem + (2 + cur) * FTILE;
#pragma unroll 1
    for (int qb = 0; qb < 2; ++qb) {
      floatx16 s, dp;
      if (active) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          s[q] = rowc[cur][0][qb * 32 + frow(q, h)];
          dp[q] = rowc[cur][1][qb * 32 + frow(q, h)];
        }
#pragma unroll
        for (int p = 0; p < 32; ++p) {
          s = fmma(Qs[foff(qb * 32 + r, 2 * p + h)], kf[p], s);    // S·scale·log2e − lse·log2e
          dp = fmma(Gs[foff(qb * 32 + r, 2 * p + h)], vf[p], dp);  // dP − δ
          if ((p & 7) == 7) __builtin_amdgcn_sched_barrier(0);   // bound the LDS-read hoisting (VGPR budget)
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          s[q] = f_exp2(s[q]);     // P
          dp[q] *= s[q];           // dS
        }
      }
      // half qb of the next Q/dO tile: issued after the score MFMAs (whose operands the register allocator partly
      // reloads from scratch, a vmcnt(0) wait that would otherwise also wait for these loads)
      if (more) {
        sq.load(Qb, ldq, (qt + 1) * 64, Lq, qb, tid);
        sg.load(Gb, lddo, (qt + 1) * 64, Lq, qb, tid);
      }
      if (active) {
#pragma unroll
        for (int p = 0; p < 16; ++p) {
          const int row = qb * 32 + frow(p, h);
          dv[0] = fmma(Gs[foff(row, r)], s[p], dv[0]);
          dv[1] = fmma(Gs[foff(row, 32 + r)], s[p], dv[1]);
          dk[0] = fmma(Qs[foff(row, r)], dp[p], dk[0]);
          dk[1] = fmma(Qs[foff(row, 32 + r)], dp[p], dk[1]);
          if ((p & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (more) {
        sq.store(smem + (cur ^ 1) * FTILE, qb, tid, c);
        sg.store(smem + (2 + (cur ^ 1)) * FTILE, qb, tid, 1.f);
      }
    }
    if (more && tid < 128) rowc[cur ^ 1][tid >> 6][tid & 63] = rc;
    __syncthreads();
  }
  if (!active) return;
  // dK = Σ dS·Q·scale; the LDS Q tiles carry scale·log2e
  const float kmul = F_LN2, vmul = 1.f;
  f_store_rows(dk, &kmul, smem + wave * 2112, dK + (long)b * Lk * lddk + hd * 64, lddk, k0, Lk, lane);
  __builtin_amdgcn_wave_barrier();
  f_store_rows(dv, &vmul, smem + wave * 2112, dV + (long)b * Lk * lddv + hd * 64, lddv, k0, Lk, lane);
}

}  // namespace

// Launchers for csrc/attention.hip's entry points (fp32 storage, D = 64, pdrop = 0); not part of the C ABI.
// Operands: 16-B aligned head slices (row strides multiples of 4 floats) — checked by the caller.
__attribute__((visibility("hidden"))) void cmhar_attn_f32m_fwd(int B, int H, int Lq, int Lk, const float* Q, long ldq,
                                                              const float* K, long ldk, const float* V, long ldv,
                                                              float* O, long ldo, float* lse, float scale,
                                                              hipStream_t st) {
  attn_fwd_f32m<<<dim3(cdiv(Lq, 128), H, B), 256, 0, st>>>(H, Lq, Lk, Q, ldq, K, ldk, V, ldv, O, ldo, lse, scale);
}

__attribute__((visibility("hidden"))) void cmhar_attn_f32m_bwd(int B, int H, int Lq, int Lk, const float* Q, long ldq,
                                                              const float* K, long ldk, const float* V, long ldv,
                                                              const float* O, long ldo, const float* dO, long lddo,
                                                              const float* lse, float* delta, float* dQ, long lddq,
                                                              float* dK, long lddk, float* dV, long lddv, float scale,
                                                              hipStream_t st) {
  attn_bwd_dq_f32m<<<dim3(cdiv(Lq, 128), H, B), 256, 0, st>>>(H, Lq, Lk, Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse,
                                                              delta, dQ, lddq, scale);
  attn_bwd_dkdv_f32m<<<dim3(cdiv(Lk, 128), H, B), 256, 0, st>>>(H, Lq, Lk, Q, ldq, K, ldk, V, ldv, dO, lddo, lse,
                                                                delta, dK, lddk, dV, lddv, scale);
}
