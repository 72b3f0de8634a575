// Fused IMU encoder forward: the whole post-LN transformer stack of IMUEncoder (models.py:85-95, 125-130; torch
// nn.TransformerEncoderLayer with d_model 128, 8 heads of 16, FF 512, ReLU, dropout) plus the final LayerNorm in ONE
// launch.
//
// The encoder runs on M = B·T tokens with T = 13 (W = 200) .. 26 (W = 400): every GEMM is a few MFLOP, so as separate
// kernels the branch was ~28 latency-bound launches per forward.  Here one workgroup owns one window: its T token rows
// stay in LDS through all layers (layer input, QKV / FFN hidden, attention output, LN1 output), weights stream
// through an LDS chunk buffer from L2 (every workgroup reads the same 770 KB per layer), and only the tensors the
// backward reads leave the CU.
//
// Numerics: bit-identical to the per-op launches (cmhar_gemm_generic, cmhar_attention_fwd's exact-f32 kernel,
// cmhar_layernorm_fwd): each GEMM output is the same k-ordered fmaf chain from 0 followed by the same epilogue
// order, and the attention rows and LayerNorm rows are the shared routines of rowops.h.
#include "common.h"
#include "rowops.h"

namespace {

constexpr int ID = 128, IH = 8, IDH = 16, IFF = 512, NT = 512;
#ifndef CMHAR_IMU_KCX
#define CMHAR_IMU_KCX 2   // chunk-size multiplier of the 128-wide weights (A/B builds)
#endif

struct IMULayerPack { CmharIMULayer l[CMHAR_IMU_MAX_LAYERS]; };

// LDS plan (floats) for at most RM token rows: Hs = layer input / LN2 output, Bg = QKV, then the out-proj output,
// then the FFN hidden, Os = attention output, then the FC2 output, H1 = LN1 output, Ws = weight chunk [N][KC].
template <int RM> struct IMUCfg {
  static constexpr int KC = RM <= 16 ? 32 : 16;       // k per staged weight chunk (RM = 32 fits 160 KiB with 16)
  static constexpr int LDD = ID + 4, LDF = IFF + 4, LDW = KC + 4;
  static constexpr int HS = 0, BG = HS + RM * LDD, OS = BG + RM * LDF, H1 = OS + RM * LDD, WS = H1 + RM * LDD;
  static constexpr int FLOATS = WS + IFF * LDW;
  // the N = 128 GEMMs (out-proj, FC2) take 2× the k per chunk in the same buffer: a chunk's L2 latency is exposed
  // once per chunk, and their chunks carry a quarter of the FMAs of the N = 512 ones
  static constexpr int kc_for(int N) { return N == ID ? CMHAR_IMU_KCX * KC : KC; }
};

// acc[i][j] = Σ_k X[rg + 4i][k] · W[cg + 128j][k], k ascending from 0 (cmhar_gemm_generic's per-output chain).
// Thread (cg = tid % 128, rg = tid / 128); W [N][K] row-major in global memory, staged per KC-wide chunk into Ws
// ([n][KC], 16-B reads along k by consecutive n: conflict-free), the next chunk's loads in flight in registers
// during the current chunk's FMAs.  X rows are LDS broadcasts (one rg per wave).
template <int RM, int N, int K>
__device__ __forceinline__ void blk_gemm(const float* __restrict__ W, const float* X, int ldx, float* Ws,
                                         float (&acc)[RM / 4][N / 128], int tid) {
  using C = IMUCfg<RM>;
  constexpr int KC = C::kc_for(N), LDW = KC + 4, NJ = N / 128, RPT = RM / 4, KQ = KC / 4, NF = N * KQ / NT;
  static_assert((N * KQ) % NT == 0 && K % KC == 0 && N * LDW <= IFF * C::LDW, "chunking");
  const int cg = tid & 127, rg = tid >> 7;
#pragma unroll
  for (int i = 0; i < RPT; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = 0.f;
  floatx4 pf[NF];
#pragma unroll
  for (int it = 0; it < NF; ++it) {
    const int e = it * NT + tid, n = e / KQ, kq = e % KQ;
    pf[it] = *(const floatx4*)(W + (long)n * K + 4 * kq);
  }
  for (int k0 = 0; k0 < K; k0 += KC) {
    __syncthreads();   // the previous chunk's readers are done; X's producers are done
#pragma unroll
    for (int it = 0; it < NF; ++it) {
      const int e = it * NT + tid, n = e / KQ, kq = e % KQ;
      *(floatx4*)(Ws + n * LDW + 4 * kq) = pf[it];
    }
    __syncthreads();
    if (k0 + KC < K) {
#pragma unroll
      for (int it = 0; it < NF; ++it) {
        const int e = it * NT + tid, n = e / KQ, kq = e % KQ;
        pf[it] = *(const floatx4*)(W + (long)n * K + k0 + KC + 4 * kq);
      }
    }
#pragma unroll 1   // (fully unrolled, the compiler hoists every chunk's LDS reads: 256 VGPRs + scratch)
    for (int kk = 0; kk < KC; kk += 4) {
      floatx4 x[RPT], w[NJ];
#pragma unroll
      for (int i = 0; i < RPT; ++i) x[i] = *(const floatx4*)(X + (rg + 4 * i) * ldx + k0 + kk);
#pragma unroll
      for (int j = 0; j < NJ; ++j) w[j] = *(const floatx4*)(Ws + (cg + 128 * j) * LDW + kk);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = fmaf(x[i][e], w[j][e], acc[i][j]);
    }
  }
}

template <int RM>
__global__ __launch_bounds__(NT) void imu_encoder_fwd_kernel(int T, int nl, const float* __restrict__ x,
                                                             IMULayerPack P, const float* __restrict__ ng,
                                                             const float* __restrict__ nb, float neps,
                                                             float* __restrict__ enc, float* __restrict__ nmu,
                                                             float* __restrict__ nrs, float scale, float pdrop,
                                                             unsigned long long seed) {
  using C = IMUCfg<RM>;
  constexpr int RPT = RM / 4, LDD = C::LDD, LDF = C::LDF;
  __shared__ __attribute__((aligned(16))) float sm[C::FLOATS];
  float* Hs = sm + C::HS;
  float* Bg = sm + C::BG;
  float* Os = sm + C::OS;
  float* H1s = sm + C::H1;
  float* Ws = sm + C::WS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = tid & 127, rg = tid >> 7;
  const int b = blockIdx.x;
  const long row0 = (long)b * T;
  for (int i = tid; i < C::WS; i += NT) sm[i] = 0.f;   // rows >= T stay zero (finite GEMM inputs, never stored)
  __syncthreads();
  for (int i = tid; i < T * ID; i += NT) {
    const int r = i / ID, c = i % ID;
    Hs[r * LDD + c] = x[(row0 + r) * ID + c];
  }
  for (int li = 0; li < nl; ++li) {
    const CmharIMULayer& L = P.l[li];
    const unsigned long long sd = seed + 7919ull * (unsigned long long)(li + 1);
    {  // qkv = h · W_qkvᵀ + b_qkv
      float acc[RPT][3];
      blk_gemm<RM, 3 * ID, ID>(L.w_qkv, Hs, LDD, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int r = rg + 4 * i, n = cg + 128 * j;
          if (r < T) {
            float v = acc[i][j];
            v += L.b_qkv[n];
            L.qkv[(row0 + r) * (3 * ID) + n] = v;
            Bg[r * LDF + n] = v;
          }
        }
    }
    __syncthreads();
    if (tid < IH * RM) {   // attention: one thread per (head, query), the exact-f32 kernel's row routine
      const int hd = tid / RM, q = tid % RM;
      const bool active = q < T;
      const int qq = active ? q : 0;
      float qv[IDH], o[IDH];
#pragma unroll
      for (int d = 0; d < IDH; ++d) { qv[d] = Bg[qq * LDF + hd * IDH + d] * scale; o[d] = 0.f; }
      float m = -INFINITY, l = 0.f;
      const unsigned bh = b * IH + hd;
      attn_row_f32<IDH>(qv, o, m, l, Bg + ID + hd * IDH, LDF, Bg + 2 * ID + hd * IDH, LDF, T, sd + 1, pdrop, bh, qq,
                        0);
      if (active) {
#pragma unroll
        for (int d = 0; d < IDH; ++d) {
          const float v = o[d] / l;
          Os[q * LDD + hd * IDH + d] = v;
          L.o[(row0 + q) * ID + hd * IDH + d] = v;
        }
        L.lse[(long)bh * T + q] = m + __logf(l);
      }
    }
    __syncthreads();
    {  // a = o · W_outᵀ + b_out  → Bg (QKV is dead)
      float acc[RPT][1];
      blk_gemm<RM, ID, ID>(L.w_out, Os, LDD, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rg + 4 * i;
        if (r < T) {
          float v = acc[i][0];
          v += L.b_out[cg];
          Bg[r * LDF + cg] = v;
        }
      }
    }
    __syncthreads();
    for (int r = wave; r < T; r += NT / 64) {   // s1 = h + drop(a), h1 = LN1(s1)
      float mu, rs;
      ln_row_fwd<float>(lane, row0 + r, ID, Hs + r * LDD, Bg + r * LDF, pdrop, sd + 2, L.s1 + (row0 + r) * ID,
                        H1s + r * LDD, L.ln1_g, L.ln1_b, L.eps1, mu, rs);
      for (int c = lane; c < ID; c += 64) L.h1[(row0 + r) * ID + c] = H1s[r * LDD + c];
      if (lane == 0) { L.mu1[row0 + r] = mu; L.rs1[row0 + r] = rs; }
    }
    __syncthreads();
    {  // fd = drop(relu(h1 · W1ᵀ + b1))  → Bg
      float acc[RPT][4];
      blk_gemm<RM, IFF, ID>(L.w_ff1, H1s, LDD, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = rg + 4 * i, n = cg + 128 * j;
          if (r < T) {
            float v = acc[i][j];
            v += L.b_ff1[n];
            v = v > 0.f ? v : 0.f;
            if (pdrop > 0.f) v *= drop_mask(sd + 3, pdrop, row0 + r, n);
            L.fd[(row0 + r) * IFF + n] = v;
            Bg[r * LDF + n] = v;
          }
        }
    }
    __syncthreads();
    {  // f2 = fd · W2ᵀ + b2  → Os
      float acc[RPT][1];
      blk_gemm<RM, ID, IFF>(L.w_ff2, Bg, LDF, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rg + 4 * i;
        if (r < T) {
          float v = acc[i][0];
          v += L.b_ff2[cg];
          Os[r * LDD + cg] = v;
        }
      }
    }
    __syncthreads();
    for (int r = wave; r < T; r += NT / 64) {   // s2 = h1 + drop(f2), h2 = LN2(s2) → Hs (next layer's input)
      float mu, rs;
      ln_row_fwd<float>(lane, row0 + r, ID, H1s + r * LDD, Os + r * LDD, pdrop, sd + 4, L.s2 + (row0 + r) * ID,
                        Hs + r * LDD, L.ln2_g, L.ln2_b, L.eps2, mu, rs);
      for (int c = lane; c < ID; c += 64) L.h2[(row0 + r) * ID + c] = Hs[r * LDD + c];
      if (lane == 0) { L.mu2[row0 + r] = mu; L.rs2[row0 + r] = rs; }
    }
    __syncthreads();
  }
  for (int r = wave; r < T; r += NT / 64) {   // enc = norm(h)
    float mu, rs;
    ln_row_fwd<float>(lane, row0 + r, ID, Hs + r * LDD, (const float*)nullptr, 0.f, 0ull, (float*)nullptr,
                      enc + (row0 + r) * ID, ng, nb, neps, mu, rs);
    if (lane == 0) { nmu[row0 + r] = mu; nrs[row0 + r] = rs; }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Backward.  Kernel 1 (one workgroup per window, all layers top-down): the per-token gradient chain — final norm
// backward, then per layer LN2 backward (+ dropout), FC2 dgrad (× ReLU′, dropout), FC1 dgrad (+ ds2), LN1 backward,
// out-proj dgrad, attention backward (exact-f32 dQ / dK / dV row routines), QKV dgrad (+ ds1) — with every GEMM a
// k-ordered fmaf chain and every row routine shared with the stand-alone kernels (bit-identical dgrads).  The
// tensors the parameter gradients need (dqkv, da, dpre, df2 and the two LayerNorms' incoming gradients) are written
// out.  Kernel 2 (grouped): every layer's four weight gradients (32 × 32 tiles, the same m-ordered chain as the
// weight-gradient GEMM) and the bias / LayerNorm-affine column sums, in one launch.
// ---------------------------------------------------------------------------------------------------------------
struct IMUGradPack { CmharIMULayerGrad g[CMHAR_IMU_MAX_LAYERS]; };

template <int RM> struct IMUBCfg {
  static constexpr int KC = RM <= 16 ? 16 : 8;        // weight rows per staged dgrad chunk
  static constexpr int LDD = ID + 4, LDF = IFF + 4;
  static constexpr int G = 0, DS = G + RM * LDD, DX = DS + RM * LDD, DH = DX + RM * LDD, BG = DH + RM * LDD,
                       DL = BG + RM * LDF, WS = DL + IH * RM;
  static constexpr int FLOATS = WS + KC * LDF;
};

// acc[i][j] = Σ_n X[rg + 4i][n] · W[n][cg + 128j], n ascending from 0 (the dgrad layout of cmhar_gemm_generic):
// W = the torch weight [NC][NOUT] (out_features × in_features), staged KC rows at a time.
template <int RM, int NOUT, int NC>
__device__ __forceinline__ void blk_dgrad(const float* __restrict__ W, const float* X, int ldx, float* Ws,
                                          float (&acc)[RM / 4][NOUT / 128], int tid) {
  using C = IMUBCfg<RM>;
  // N = 128-wide weights: rows of 132 floats, so 2× (RM = 32) to 2× (RM = 16) the rows per chunk in the same buffer
  constexpr int KC = NOUT == ID ? CMHAR_IMU_KCX * C::KC : C::KC, LDW = NOUT + 4, NJ = NOUT / 128, RPT = RM / 4, NQ = NOUT / 4;
  constexpr int TOT = KC * NQ, NF = (TOT + NT - 1) / NT;
  static_assert(NC % KC == 0 && KC % 4 == 0 && KC * LDW <= C::KC * C::LDF, "chunking");
  const int cg = tid & 127, rg = tid >> 7;
#pragma unroll
  for (int i = 0; i < RPT; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = 0.f;
  floatx4 pf[NF];
#pragma unroll
  for (int it = 0; it < NF; ++it) {
    const int e = it * NT + tid;
    if (e < TOT) pf[it] = *(const floatx4*)(W + (long)(e / NQ) * NOUT + 4 * (e % NQ));
  }
  for (int n0 = 0; n0 < NC; n0 += KC) {
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NF; ++it) {
      const int e = it * NT + tid;
      if (e < TOT) *(floatx4*)(Ws + (e / NQ) * LDW + 4 * (e % NQ)) = pf[it];
    }
    __syncthreads();
    if (n0 + KC < NC) {
#pragma unroll
      for (int it = 0; it < NF; ++it) {
        const int e = it * NT + tid;
        if (e < TOT) pf[it] = *(const floatx4*)(W + (long)(n0 + KC + e / NQ) * NOUT + 4 * (e % NQ));
      }
    }
#pragma unroll 1
    for (int nn = 0; nn < KC; nn += 4) {
      floatx4 x[RPT];
#pragma unroll
      for (int i = 0; i < RPT; ++i) x[i] = *(const floatx4*)(X + (rg + 4 * i) * ldx + n0 + nn);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float w[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) w[j] = Ws[(nn + e) * LDW + cg + 128 * j];
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = fmaf(x[i][e], w[j], acc[i][j]);
      }
    }
  }
}

// LayerNorm backward of the rows < T (one wave per row, two columns per lane: N = 128) as the stand-alone
// ln_bwd_kernel<float, 2>: dy from LDS (dyl), x from the saved pre-norm tensor (global).  out(r, c, v) receives
// each column's gradient.
template <typename F>
__device__ __forceinline__ void ln_rows_bwd(int T, long row0, int wave, int lane, const float* dyl, int lddy,
                                            const float* __restrict__ hs, const float* __restrict__ mu,
                                            const float* __restrict__ rs, const float* __restrict__ gamma, F out) {
  for (int r = wave; r < T; r += NT / 64) {
    float pd[2], ph[2], ag[2] = {0.f, 0.f}, ab[2] = {0.f, 0.f}, gx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      pd[i] = dyl[r * lddy + lane + 64 * i];
      ph[i] = hs[(row0 + r) * ID + lane + 64 * i];
    }
    ln_row_bwd<2>(lane, ID, pd, ph, mu[row0 + r], rs[row0 + r], gamma, ag, ab, gx);
#pragma unroll
    for (int i = 0; i < 2; ++i) out(r, lane + 64 * i, gx[i]);
  }
}

template <int RM>
__global__ __launch_bounds__(NT) void imu_encoder_bwd_kernel(int T, int nl, IMULayerPack P, IMUGradPack Gp,
                                                             const float* __restrict__ ng,
                                                             const float* __restrict__ nmu,
                                                             const float* __restrict__ nrs,
                                                             const float* __restrict__ denc, float* __restrict__ dx,
                                                             float scale, float pdrop, unsigned long long seed) {
  using C = IMUBCfg<RM>;
  constexpr int RPT = RM / 4, LDD = C::LDD, LDF = C::LDF;
  __shared__ __attribute__((aligned(16))) float sm[C::FLOATS];
  float* G = sm + C::G;
  float* DS = sm + C::DS;
  float* DX = sm + C::DX;
  float* DH = sm + C::DH;
  float* BG = sm + C::BG;
  float* DL = sm + C::DL;
  float* Ws = sm + C::WS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = tid & 127, rg = tid >> 7;
  const int b = blockIdx.x;
  const long row0 = (long)b * T;
  for (int i = tid; i < C::WS; i += NT) sm[i] = 0.f;
  __syncthreads();
  for (int i = tid; i < T * ID; i += NT) {   // d_enc rows → DX (staging for the final norm's backward)
    const int r = i / ID, c = i % ID;
    DX[r * LDD + c] = denc[(row0 + r) * ID + c];
  }
  __syncthreads();
  // final norm: G = norm_bwd(d_enc) over the last layer's output
  ln_rows_bwd(T, row0, wave, lane, DX, LDD, P.l[nl - 1].h2, nmu, nrs, ng,
              [&](int r, int c, float v) { G[r * LDD + c] = v; });
  for (int li = nl - 1; li >= 0; --li) {
    const CmharIMULayer& L = P.l[li];
    const CmharIMULayerGrad& Q = Gp.g[li];
    const unsigned long long sd = seed + 7919ull * (unsigned long long)(li + 1);
    const float* hin = li > 0 ? P.l[li - 1].h2 : nullptr;
    (void)hin;
    __syncthreads();
    // LN2: ds2 → DS, df2 = ds2 · mask → DX (+ global); the incoming gradient is LN2's dy (global, for dγ / dβ)
    for (int i = tid; i < T * ID; i += NT) {
      const int r = i / ID, c = i % ID;
      Q.gln2[(row0 + r) * ID + c] = G[r * LDD + c];
    }
    ln_rows_bwd(T, row0, wave, lane, G, LDD, L.s2, L.mu2, L.rs2, L.ln2_g, [&](int r, int c, float v) {
      DS[r * LDD + c] = v;
      const float d = v * drop_mask(sd + 4, pdrop, row0 + r, c);
      DX[r * LDD + c] = d;
      Q.df2[(row0 + r) * ID + c] = d;
    });
    __syncthreads();
    {  // dpre = drop(relu′(fd) · (df2 · W2))  → BG
      float acc[RPT][4];
      blk_dgrad<RM, IFF, ID>(L.w_ff2, DX, LDD, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = rg + 4 * i, n = cg + 128 * j;
          if (r < T) {
            float v = acc[i][j];
            v = L.fd[(row0 + r) * IFF + n] > 0.f ? v : 0.f;
            if (pdrop > 0.f) v *= drop_mask(sd + 3, pdrop, row0 + r, n);
            BG[r * LDF + n] = v;
            Q.dpre[(row0 + r) * IFF + n] = v;
          }
        }
    }
    __syncthreads();
    {  // dh1 = dpre · W1 + ds2  → DH (+ global: LN1's dy)
      float acc[RPT][1];
      blk_dgrad<RM, ID, IFF>(L.w_ff1, BG, LDF, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rg + 4 * i;
        if (r < T) {
          float v = acc[i][0];
          v += DS[r * LDD + cg];
          DH[r * LDD + cg] = v;
          Q.gln1[(row0 + r) * ID + cg] = v;
        }
      }
    }
    __syncthreads();
    // LN1: ds1 → DS, da = ds1 · mask → DX (+ global)
    ln_rows_bwd(T, row0, wave, lane, DH, LDD, L.s1, L.mu1, L.rs1, L.ln1_g, [&](int r, int c, float v) {
      DS[r * LDD + c] = v;
      const float d = v * drop_mask(sd + 2, pdrop, row0 + r, c);
      DX[r * LDD + c] = d;
      Q.da[(row0 + r) * ID + c] = d;
    });
    __syncthreads();
    {  // do = da · W_out  → DH
      float acc[RPT][1];
      blk_dgrad<RM, ID, ID>(L.w_out, DX, LDD, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rg + 4 * i;
        if (r < T) DH[r * LDD + cg] = acc[i][0];
      }
    }
    // stage qkv (the forward's saved projection) → BG; delta = rowsum(dO ∘ O) per (head, query) → DL
    for (int i = tid; i < T * 3 * ID; i += NT) {
      const int r = i / (3 * ID), c = i % (3 * ID);
      BG[r * LDF + c] = L.qkv[(row0 + r) * (3 * ID) + c];
    }
    __syncthreads();
    if (tid < IH * RM) {
      const int hd = tid / RM, q = tid % RM;
      float delta = 0.f;
      if (q < T) {
#pragma unroll
        for (int d = 0; d < IDH; ++d) {
          const float g = DH[q * LDD + hd * IDH + d];
          delta = fmaf(g, L.o[(row0 + q) * ID + hd * IDH + d], delta);   // as attn_bwd_dq_f32
        }
      }
      DL[hd * RM + q] = delta;
    }
    __syncthreads();
    // attention backward: threads [0, 8·RM) one query row each (dQ), [8·RM, 16·RM) one key row each (dK, dV)
    float r0[IDH], r1[IDH];
    int arow = -1, acol = 0;
    if (tid < IH * RM) {
      const int hd = tid / RM, q = tid % RM;
      const int qq = q < T ? q : 0;
      const unsigned bh = b * IH + hd;
      float qv[IDH], g[IDH];
#pragma unroll
      for (int d = 0; d < IDH; ++d) {
        qv[d] = BG[qq * LDF + hd * IDH + d] * scale;
        g[d] = DH[qq * LDD + hd * IDH + d];
        r0[d] = 0.f;
      }
      attn_row_dq_f32<IDH>(qv, g, L.lse[(long)bh * T + qq], DL[hd * RM + qq], r0, BG + ID + hd * IDH, LDF,
                           BG + 2 * ID + hd * IDH, LDF, T, sd + 1, pdrop, bh, qq, 0);
      if (q < T) { arow = q; acol = hd * IDH; }
#pragma unroll
      for (int d = 0; d < IDH; ++d) r0[d] *= scale;
    } else if (tid < 2 * IH * RM) {
      const int t = tid - IH * RM, hd = t / RM, k = t % RM;
      const int kk = k < T ? k : 0;
      const unsigned bh = b * IH + hd;
      float kv[IDH], vv[IDH];
#pragma unroll
      for (int d = 0; d < IDH; ++d) {
        kv[d] = BG[kk * LDF + ID + hd * IDH + d];
        vv[d] = BG[kk * LDF + 2 * ID + hd * IDH + d];
        r0[d] = 0.f;
        r1[d] = 0.f;
      }
      attn_row_dkdv_f32<IDH>(kv, vv, r0, r1, BG + hd * IDH, LDF, scale, DH + hd * IDH, LDD, L.lse + (long)bh * T,
                             DL + hd * RM, T, sd + 1, pdrop, bh, 0, kk);
      if (k < T) { arow = k; acol = ID + hd * IDH; }
    }
    __syncthreads();   // every reader of qkv is done: dqkv → BG (+ global)
    if (arow >= 0) {
#pragma unroll
      for (int d = 0; d < IDH; ++d) {
        BG[arow * LDF + acol + d] = r0[d];
        Q.dqkv[(row0 + arow) * (3 * ID) + acol + d] = r0[d];
      }
      if (acol >= ID) {
#pragma unroll
        for (int d = 0; d < IDH; ++d) {
          BG[arow * LDF + acol + ID + d] = r1[d];
          Q.dqkv[(row0 + arow) * (3 * ID) + acol + ID + d] = r1[d];
        }
      }
    }
    __syncthreads();
    {  // dh = dqkv · W_qkv + ds1  → G (the next layer down's incoming gradient)
      float acc[RPT][1];
      blk_dgrad<RM, ID, 3 * ID>(L.w_qkv, BG, LDF, Ws, acc, tid);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rg + 4 * i;
        if (r < T) {
          float v = acc[i][0];
          v += DS[r * LDD + cg];
          G[r * LDD + cg] = v;
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < T * ID; i += NT) {
    const int r = i / ID, c = i % ID;
    dx[(row0 + r) * ID + c] = G[r * LDD + c];
  }
}

// Kernel 2.  Blocks [0, 192·nl): weight-gradient tiles (per layer: QKV 12×4, out 4×4, FC1 16×4, FC2 4×16 tiles of
// 32 × 32); then per layer 44 column-sum items of 32 columns (biases of qkv 12, out 4, ff1 16, ff2 4; LN1 and LN2
// affine 4 each), then the final norm's affine (4).  dW[n][k] = Σ_m dY[m][n] · X[m][k], m ascending from 0 (the weight-gradient GEMM chain).
constexpr int WG_TILES = 192, WG_SUMS = 44, WG_FINAL = 4, WT = 32, WKT = 32;

struct WgJob { const float* dy; int ldy; const float* x; int ldx; float* dw; int N, K; };

__device__ __forceinline__ void wgrad_tile(int M, const WgJob& j, int tile, float (*As)[WT + 4], float (*Bs)[WT + 4]) {
  const int tn = j.K / WT;
  const int n0 = (tile / tn) * WT, k0 = (tile % tn) * WT;
  const int tid = threadIdx.x, tr = tid / 16, tc = tid % 16;
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  // per chunk of WKT token rows: thread loads 4 dY and 4 X elements (rows tid / 8 .. , 4 consecutive columns)
  const int lr = tid / 8, lc = (tid % 8) * 4;
  floatx4 pa, pb;
  auto load = [&](int m0) {
    const int m = m0 + lr;
    if (m < M) {
      pa = *(const floatx4*)(j.dy + (long)m * j.ldy + n0 + lc);
      pb = *(const floatx4*)(j.x + (long)m * j.ldx + k0 + lc);
    } else {
      pa = floatx4{0.f, 0.f, 0.f, 0.f};
      pb = pa;
    }
  };
  load(0);
  for (int m0 = 0; m0 < M; m0 += WKT) {
    __syncthreads();
    *(floatx4*)&As[lr][lc] = pa;
    *(floatx4*)&Bs[lr][lc] = pb;
    __syncthreads();
    if (m0 + WKT < M) load(m0 + WKT);
    const int mn = min(WKT, M - m0);
    for (int mm = 0; mm < mn; ++mm) {
      const float a0 = As[mm][tr], a1 = As[mm][tr + 16], b0 = Bs[mm][tc], b1 = Bs[mm][tc + 16];
      acc[0][0] = fmaf(a0, b0, acc[0][0]);
      acc[0][1] = fmaf(a0, b1, acc[0][1]);
      acc[1][0] = fmaf(a1, b0, acc[1][0]);
      acc[1][1] = fmaf(a1, b1, acc[1][1]);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) j.dw[(long)(n0 + tr + 16 * i) * j.K + k0 + tc + 16 * jj] = acc[i][jj];
}

// Column sums over the M token rows for 32 columns c0 .. c0+31: out[c] = Σ_m dy[m][c] (bias), or with hs: γ[c] =
// Σ_m dy·x̂, β[c] = Σ_m dy (LayerNorm affine; x̂ = (h − μ)·r).  8 row groups (m ≡ g mod 8, 32 consecutive columns
// each: 128-B rows) keep 8× the loads in flight of one thread per column; partials combined in group order.
__device__ __forceinline__ void colsum_item(int M, const float* __restrict__ dy, int ldy, int c0,
                                            float* __restrict__ out, const float* __restrict__ hs,
                                            const float* __restrict__ mu, const float* __restrict__ rs,
                                            float* __restrict__ out2, float (*red)[2][32]) {
  const int c = threadIdx.x & 31, g = threadIdx.x >> 5;
  float s = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int m = g; m < M; m += 8) {
    const float d = dy[(long)m * ldy + c0 + c];
    if (hs) s2 = fmaf(d, (hs[(long)m * ID + c0 + c] - mu[m]) * rs[m], s2);
    s += d;
  }
  red[g][0][c] = s;
  red[g][1][c] = s2;
  __syncthreads();
  if (g == 0) {
    float t = 0.f, t2 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) { t += red[k][0][c]; t2 += red[k][1][c]; }
    if (hs) { out[c0 + c] = t2; out2[c0 + c] = t; }
    else out[c0 + c] = t;
  }
}

__global__ __launch_bounds__(256) void imu_encoder_wgrad_kernel(int M, int nl, const float* __restrict__ x0,
                                                                IMULayerPack P, IMUGradPack Gp,
                                                                const float* __restrict__ denc,
                                                                const float* __restrict__ nmu,
                                                                const float* __restrict__ nrs,
                                                                float* __restrict__ dng, float* __restrict__ dnb) {
  __shared__ __attribute__((aligned(16))) float As[WKT][WT + 4];
  __shared__ __attribute__((aligned(16))) float Bs[WKT][WT + 4];
  const int bid = blockIdx.x;
  if (bid < nl * WG_TILES) {
    const int li = bid / WG_TILES, t = bid % WG_TILES;
    const CmharIMULayer& L = P.l[li];
    const CmharIMULayerGrad& Q = Gp.g[li];
    const float* hin = li > 0 ? P.l[li - 1].h2 : x0;
    WgJob j;
    int tile;
    if (t < 48)       { j = {Q.dqkv, 3 * ID, hin, ID, Q.dw_qkv, 3 * ID, ID}; tile = t; }
    else if (t < 64)  { j = {Q.da, ID, L.o, ID, Q.dw_out, ID, ID}; tile = t - 48; }
    else if (t < 128) { j = {Q.dpre, IFF, L.h1, ID, Q.dw_ff1, IFF, ID}; tile = t - 64; }
    else              { j = {Q.df2, ID, L.fd, IFF, Q.dw_ff2, ID, IFF}; tile = t - 128; }
    wgrad_tile(M, j, tile, As, Bs);
    return;
  }
  __shared__ float red[8][2][32];
  const int s = bid - nl * WG_TILES;
  if (s < nl * WG_SUMS) {
    const int li = s / WG_SUMS, it = s % WG_SUMS;
    const CmharIMULayer& L = P.l[li];
    const CmharIMULayerGrad& Q = Gp.g[li];
    if (it < 12)      colsum_item(M, Q.dqkv, 3 * ID, 32 * it, Q.db_qkv, nullptr, nullptr, nullptr, nullptr, red);
    else if (it < 16) colsum_item(M, Q.da, ID, 32 * (it - 12), Q.db_out, nullptr, nullptr, nullptr, nullptr, red);
    else if (it < 32) colsum_item(M, Q.dpre, IFF, 32 * (it - 16), Q.db_ff1, nullptr, nullptr, nullptr, nullptr, red);
    else if (it < 36) colsum_item(M, Q.df2, ID, 32 * (it - 32), Q.db_ff2, nullptr, nullptr, nullptr, nullptr, red);
    else if (it < 40) colsum_item(M, Q.gln1, ID, 32 * (it - 36), Q.dln1_g, L.s1, L.mu1, L.rs1, Q.dln1_b, red);
    else              colsum_item(M, Q.gln2, ID, 32 * (it - 40), Q.dln2_g, L.s2, L.mu2, L.rs2, Q.dln2_b, red);
    return;
  }
  const int f = s - nl * WG_SUMS;
  colsum_item(M, denc, ID, 32 * f, dng, P.l[nl - 1].h2, nmu, nrs, dnb, red);
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int cmhar_imu_encoder_fwd(int B, int T, int D, int H, int FF, int nlayers, const float* x,
                                     const CmharIMULayer* layers, const float* norm_g, const float* norm_b,
                                     float norm_eps, float* enc, float* norm_mu, float* norm_rs, float scale,
                                     float pdrop, unsigned long long seed, hipStream_t st) {
  if (B <= 0) return 0;
  if (D != ID || H != IH || FF != IFF || T < 1 || T > 32 || nlayers < 0 || nlayers > CMHAR_IMU_MAX_LAYERS ||
      !x || !layers || !norm_g || !norm_b || !enc || !norm_mu || !norm_rs)
    return -1;
  IMULayerPack P;
  for (int i = 0; i < nlayers; ++i) {
    const CmharIMULayer& L = layers[i];
    const void* need[] = {L.w_qkv, L.b_qkv, L.w_out, L.b_out, L.ln1_g, L.ln1_b, L.w_ff1, L.b_ff1, L.w_ff2, L.b_ff2,
                          L.ln2_g, L.ln2_b, L.qkv, L.o, L.lse, L.s1, L.mu1, L.rs1, L.h1, L.fd, L.s2, L.mu2, L.rs2,
                          L.h2};
    for (const void* p : need)
      if (!p) return -1;
    if (!al16(L.w_qkv) || !al16(L.w_out) || !al16(L.w_ff1) || !al16(L.w_ff2)) return -2;   // 16-B weight loads
    P.l[i] = L;
  }
  if (T <= 16)
    imu_encoder_fwd_kernel<16><<<B, NT, 0, st>>>(T, nlayers, x, P, norm_g, norm_b, norm_eps, enc, norm_mu, norm_rs,
                                                 scale, pdrop, seed);
  else
    imu_encoder_fwd_kernel<32><<<B, NT, 0, st>>>(T, nlayers, x, P, norm_g, norm_b, norm_eps, enc, norm_mu, norm_rs,
                                                 scale, pdrop, seed);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_imu_encoder_bwd(int B, int T, int D, int H, int FF, int nlayers, const float* x,
                                     const CmharIMULayer* layers, const CmharIMULayerGrad* grads,
                                     const float* norm_g, const float* norm_mu, const float* norm_rs,
                                     const float* d_enc, float* dnorm_g, float* dnorm_b, float* dx, float scale,
                                     float pdrop, unsigned long long seed, hipStream_t st) {
  if (B <= 0) return 0;
  if (D != ID || H != IH || FF != IFF || T < 1 || T > 32 || nlayers < 1 || nlayers > CMHAR_IMU_MAX_LAYERS || !x ||
      !layers || !grads || !norm_g || !norm_mu || !norm_rs || !d_enc || !dnorm_g || !dnorm_b || !dx)
    return -1;
  IMULayerPack P;
  IMUGradPack G;
  for (int i = 0; i < nlayers; ++i) {
    const CmharIMULayer& L = layers[i];
    const CmharIMULayerGrad& Q = grads[i];
    const void* need[] = {L.w_qkv, L.w_out, L.ln1_g, L.w_ff1, L.w_ff2, L.ln2_g, L.qkv, L.o, L.lse, L.s1, L.mu1,
                          L.rs1, L.h1, L.fd, L.s2, L.mu2, L.rs2, L.h2, Q.dqkv, Q.da, Q.dpre, Q.df2, Q.gln1,
                          Q.gln2, Q.dw_qkv, Q.db_qkv, Q.dw_out, Q.db_out, Q.dln1_g, Q.dln1_b, Q.dw_ff1, Q.db_ff1,
                          Q.dw_ff2, Q.db_ff2, Q.dln2_g, Q.dln2_b};
    for (const void* p : need)
      if (!p) return -1;
    // 16-B loads: weights, the saved / gradient token tensors (row widths are multiples of 4 floats)
    const void* vec[] = {L.w_qkv, L.w_out, L.w_ff1, L.w_ff2, L.o, L.h1, L.fd, L.h2, Q.dqkv, Q.da, Q.dpre, Q.df2};
    for (const void* p : vec)
      if (!al16(p)) return -2;
    P.l[i] = L;
    G.g[i] = Q;
  }
  if (!al16(x)) return -2;
  if (T <= 16)
    imu_encoder_bwd_kernel<16><<<B, NT, 0, st>>>(T, nlayers, P, G, norm_g, norm_mu, norm_rs, d_enc, dx, scale, pdrop,
                                                 seed);
  else
    imu_encoder_bwd_kernel<32><<<B, NT, 0, st>>>(T, nlayers, P, G, norm_g, norm_mu, norm_rs, d_enc, dx, scale, pdrop,
                                                 seed);
  CMHAR_CHECK_LAUNCH();
  imu_encoder_wgrad_kernel<<<nlayers * (WG_TILES + WG_SUMS) + WG_FINAL, 256, 0, st>>>(B * T, nlayers, x, P, G, d_enc, norm_mu,
                                                                                norm_rs, dnorm_g, dnorm_b);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
