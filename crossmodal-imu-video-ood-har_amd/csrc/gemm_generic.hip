// Generic strided GEMM with fp32 accumulation.
//
// Used for (a) the exact-fp32 parity mode of every Linear on the path and (b) the small, latency-bound
// GEMMs of the IMU encoder / projection heads (M = batch*13 or batch rows), where an MFMA tile would idle.
// C[m,n] = epilogue( sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] ), batched over blockIdx.z.
//
// Two kernels, ONE numerics: every output is the k-ordered fmaf chain from 0.  The VALU kernel does it with fmaf;
// the f32-input MFMA (v_mfma_f32_32x32x2_f32, 157 TF/s, bitwise the k-ordered fmaf chain: lanes 0-31 carry k, lanes
// 32-63 carry k+1, applied in that order) does it for every f32 GEMM with >= 64 output tiles of 128², so the fp32
// parity mode's VideoMAE GEMMs move to the matrix cores with bit-identical results.
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, TK = 32, NTH = 256;   // default tile; T = 32 for grids of few 64² tiles
#ifndef CMHAR_SMALL_KT
#define CMHAR_SMALL_KT 64    // K-tile of the few-tile (T = 32) kernel when K >= it (A/B: tools/debug/imu_kt_ab.sh)
#endif

// The GEMMs this kernel serves are small (tens of blocks) with K up to a few thousand, so a K-step is bounded by
// memory LATENCY, not bandwidth: tile k+1 is loaded into registers while tile k is consumed from LDS (double-
// buffered LDS, one barrier per K-step), so each step pays compute + one overlapped fetch.
template <typename TIn, int T, int KT = TK>
struct GenStage {
  static constexpr int TK = KT;
  static constexpr int PER = T * TK / NTH;      // A and B elements staged per thread per K-tile
  float a[PER], b[PER];
  __device__ __forceinline__ void load(const TIn* __restrict__ A, long sam, long sak, const TIn* __restrict__ B,
                                       long sbk, long sbn, int M, int N, int K, int bm, int bn, int k0, int tid) {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = it * NTH + tid;
      int mm, kk;
      if (sak == 1) { mm = i / TK; kk = i % TK; } else { kk = i / T; mm = i % T; }
      const int gm = bm + mm, gk = k0 + kk;
      a[it] = (gm < M && gk < K) ? to_f<TIn>(A[gm * sam + gk * sak]) : 0.f;
      int nn, kb;
      if (sbn == 1) { kb = i / T; nn = i % T; } else { nn = i / TK; kb = i % TK; }
      const int gn = bn + nn, gkb = k0 + kb;
      b[it] = (gn < N && gkb < K) ? to_f<TIn>(B[gkb * sbk + gn * sbn]) : 0.f;
    }
  }
  __device__ __forceinline__ void store(float (*As)[T + 4], float (*Bs)[T + 4], long sak, long sbn, int tid) const {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = it * NTH + tid;
      int mm, kk;
      if (sak == 1) { mm = i / TK; kk = i % TK; } else { kk = i / T; mm = i % T; }
      As[kk][mm] = a[it];
      int nn, kb;
      if (sbn == 1) { kb = i / T; nn = i % T; } else { nn = i / TK; kb = i % TK; }
      Bs[kb][nn] = b[it];
    }
  }
};

// T x T output tile, 16 x 16 threads with (T/16)² outputs each.  Every output is one fmaf chain over k = 0..K-1 in
// order whatever T is, so the two tile sizes give bit-identical results (T = 32 quadruples the workgroups of the
// IMU encoder's few-tile GEMMs and quarters each one's K-loop FMA count).
// KT: K-tile.  The IMU encoder's few-tile GEMMs (T = 32) take KT = CMHAR_SMALL_KT = 64 when K >= 64: their K-steps
// are bound by the global-load latency, so more k per step exposes fewer latencies (same per-output fmaf chain).
// Measured (tools/debug/imu_kt_ab.sh, one box): standalone KT 32 → 128 cut the GEMMs 21.5 → 15.9 µs, but inside the
// bench step, where these workgroups only fill gaps beside the video kernels, KT = 64 gives the least IMU GEMM time
// (2.7 ms/step vs 3.2 at 32 and 3.9 at 128); the step's wall time is the same for all three.
template <typename TIn, typename TOut, int T = TM, int KT = TK>
__global__ __launch_bounds__(NTH) void gemm_generic_kernel(
    int M, int N, int K, const TIn* __restrict__ A, long sam, long sak, long sAb, const TIn* __restrict__ B,
    long sbk, long sbn, long sBb, TOut* __restrict__ C, long ldc, long sCb, Epilogue e) {
  constexpr int R = T / 16, TK = KT;
  __shared__ float As[2][TK][T + 4];
  __shared__ float Bs[2][TK][T + 4];
  const int tid = threadIdx.x;
  const int bm = blockIdx.y * T, bn = blockIdx.x * T;
  A += blockIdx.z * sAb;
  B += blockIdx.z * sBb;
  C += blockIdx.z * sCb;
  const int tr = tid / 16, tc = tid % 16;   // 16x16 threads, R x R outputs each
  float acc[R][R] = {};
  const int nk = (K + TK - 1) / TK;
  GenStage<TIn, T, KT> st;
  st.load(A, sam, sak, B, sbk, sbn, M, N, K, bm, bn, 0, tid);
  st.store(As[0], Bs[0], sak, sbn, tid);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) st.load(A, sam, sak, B, sbk, sbn, M, N, K, bm, bn, (t + 1) * TK, tid);
#pragma unroll 8
    for (int kk = 0; kk < TK; ++kk) {
      float a[R], b[R];
#pragma unroll
      for (int i = 0; i < R; ++i) { a[i] = As[cur][kk][tr + 16 * i]; b[i] = Bs[cur][kk][tc + 16 * i]; }
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    if (t + 1 < nk) st.store(As[cur ^ 1], Bs[cur ^ 1], sak, sbn, tid);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int m = bm + tr + 16 * i, n = bn + tc + 16 * j;
      if (m < M && n < N) epilogue_store<TOut>(e, C, ldc, m, n, acc[i][j]);
    }
}

// ---- f32 MFMA kernel --------------------------------------------------------------------------------------------
// (64·WM) x (64·WN) output tile per block of WM x WN waves, 32-k steps; wave (wm, wn) owns a 64 x 64 quadrant = 2 x 2
// blocks of 32 x 32 accumulators (64 acc VGPRs).  Operand panels are staged global → registers → LDS as [k][row]
// (the MFMA reads one f32 per lane: row l&31 of k = 2p + (l>>5)), double-buffered with one barrier per k-step; the
// next panel's global loads are in flight during the current one's 64 MFMAs per wave.  Tiles are walked in groups
// of FGROUP tile-rows (every group column-by-column) in XCD-contiguous chunks, so the blocks co-resident on one XCD
// share A and B panels through its L2 instead of streaming them from the Infinity Cache.
// 16-k steps at 3 blocks per CU: 5 % faster than 32-k steps at 2 (double-buffered panels 33 KB vs 66 KB per block;
// tools/debug/gemm_ab.py --dtype fp32, bit-identical results)
#ifndef CMHAR_F32_BK
#define CMHAR_F32_BK 16
#endif
#ifndef CMHAR_F32_OCC
#define CMHAR_F32_OCC 3
#endif
constexpr int FK = CMHAR_F32_BK;
#ifndef CMHAR_F32_WM
#define CMHAR_F32_WM 2
#endif
#ifndef CMHAR_F32_GROUP
#define CMHAR_F32_GROUP 8
#endif
constexpr int FWM = CMHAR_F32_WM, FWN = 2, FGROUP = CMHAR_F32_GROUP;

// One ROWS-row x 32-k operand panel.  KC: element (r, k) at P[r*ld + k] (k contiguous; 16-B loads along k, written
// transposed); else at P[k*ld + r] (rows contiguous; 16-B loads and 16-B LDS writes along r).
template <bool KC, int ROWS, int NT>
struct F32Panel {
  static constexpr int LD = KC ? ROWS + 1 : ROWS + 4;   // LDS stride of one k row (floats): +1 spreads the
                                                        // transposed scalar writes over banks, +4 keeps 16-B writes aligned
  static constexpr int FLOATS = FK * LD;
  static constexpr int PER = ROWS * FK / 4 / NT;        // float4 per thread
  static constexpr int RQ = ROWS / 4, KQ = FK / 4;
  floatx4 v[PER];
  __device__ __forceinline__ void load(const float* __restrict__ P, long ld, int R, int K, int r0, int k0, int tid) {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = it * NT + tid;
      int r, k;
      if (KC) { r = i / KQ; k = (i % KQ) * 4; } else { k = i / RQ; r = (i % RQ) * 4; }
      const int gr = r0 + r, gk = k0 + k;
      // K (KC) or R (!KC) is a multiple of 4 (host-checked): a 16-B vector is wholly inside or wholly outside
      const bool ok = gr < R && gk < K;
      const float* src = KC ? P + (long)gr * ld + gk : P + (long)gk * ld + gr;
      v[it] = ok ? *(const floatx4*)src : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ S, int tid) const {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = it * NT + tid;
      if (KC) {
        const int r = i / KQ, k = (i % KQ) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) S[(k + j) * LD + r] = v[it][j];
      } else {
        *(floatx4*)(S + (i / RQ) * LD + (i % RQ) * 4) = v[it];
      }
    }
  }
};

template <int WM, int WN, bool A_KC, bool B_KC, typename OutT>
__global__ __launch_bounds__(64 * WM * WN, WM * WN == 4 ? CMHAR_F32_OCC : 1) void gemm_f32_mfma_kernel(
    int M, int N, int K, const float* __restrict__ A, long lda, long sAb, const float* __restrict__ B, long ldb,
    long sBb, OutT* __restrict__ C, long ldc, long sCb, Epilogue e) {
  constexpr int BM = 64 * WM, BN = 64 * WN, NT = 64 * WM * WN;
  typedef F32Panel<A_KC, BM, NT> PA;
  typedef F32Panel<B_KC, BN, NT> PB;
  constexpr int ELD = 65;                              // epilogue staging: 32 rows x 64 (+1) per wave
  constexpr int PANELS = 2 * (PA::FLOATS + PB::FLOATS), STAGE = WM * WN * 32 * ELD;
  __shared__ float smem[PANELS > STAGE ? PANELS : STAGE];
  float* const As0 = smem;                             // panel buffers: A[0], A[1], B[0], B[1]
  float* const Bs0 = smem + 2 * PA::FLOATS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN, r = lane & 31, h = lane >> 5;
  // XCD-contiguous, row-grouped tile order
  const int tn_count = (N + BN - 1) / BN, tm_count = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = FGROUP * tn_count, g = t / per_group;
  const int gm = min(FGROUP, tm_count - g * FGROUP), tin = t - g * per_group;
  const int bm = (g * FGROUP + tin % gm) * BM, bn = (tin / gm) * BN;
  A += blockIdx.z * sAb;
  B += blockIdx.z * sBb;
  C += blockIdx.z * sCb;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int nk = (K + FK - 1) / FK;
  PA pa;
  PB pb;
  pa.load(A, lda, M, K, bm, 0, tid);
  pb.load(B, ldb, N, K, bn, 0, tid);
  pa.store(As0, tid);
  pb.store(Bs0, tid);
  __syncthreads();
  const int ao = wm * 64 + r, bo = wn * 64 + r;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      pa.load(A, lda, M, K, bm, (kt + 1) * FK, tid);
      pb.load(B, ldb, N, K, bn, (kt + 1) * FK, tid);
    }
    const float* as = As0 + cur * PA::FLOATS;
    const float* bs = Bs0 + cur * PB::FLOATS;
#pragma unroll
    for (int p = 0; p < FK / 2; ++p) {
      const int k = 2 * p + h;
      const float a0 = as[k * PA::LD + ao], a1 = as[k * PA::LD + ao + 32];
      const float b0 = bs[k * PB::LD + bo], b1 = bs[k * PB::LD + bo + 32];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      pa.store(As0 + (cur ^ 1) * PA::FLOATS, tid);
      pb.store(Bs0 + (cur ^ 1) * PB::FLOATS, tid);
    }
    __syncthreads();
  }
  // Epilogue per wave, one 32-row half of its quadrant at a time, staged through a wave-private LDS region (C/D map
  // of the 32x32 forms: col = lane&31, row = (q&3) + 8(q>>2) + 4(lane>>5)) so that each lane applies the epilogue to
  // one column of a 256-B row — coalesced C / residual / aux traffic, and no dynamic indexing of the accumulators
  // (the epilogue body is too large to unroll 64 times).  The loop's last barrier freed the panels.
  float* const st = smem + w * 32 * ELD;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) st[((q & 3) + 8 * (q >> 2) + 4 * h) * ELD + 32 * j + r] = acc[i][j][q];
    __builtin_amdgcn_wave_barrier();   // wave-private region: one wave's LDS ops complete in order
    const int m0 = bm + wm * 64 + 32 * i, n = bn + wn * 64 + lane;
#pragma unroll 4
    for (int row = 0; row < 32; ++row)
      if (m0 + row < M && n < N) epilogue_store<OutT>(e, C, ldc, m0 + row, n, st[row * ELD + lane]);
    __builtin_amdgcn_wave_barrier();
  }
}

// Split-K combine: C = epilogue(Σ_s P[s]) in a fixed split order (deterministic).
template <typename TOut>
__global__ __launch_bounds__(256) void generic_splitk_reduce(int M, int N, int S, const float* __restrict__ P,
                                                             TOut* __restrict__ C, long ldc, Epilogue e) {
  const long MN = (long)M * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < MN; i += (long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s) acc += P[s * MN + i];
    epilogue_store<TOut>(e, C, ldc, (int)(i / N), (int)(i % N), acc);
  }
}

}  // namespace

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// The f32 MFMA kernel takes f32 operands whose contiguous dimension allows 16-B loads: that dimension a multiple of
// 4 elements, the other stride and the batch stride multiples of 4, 16-B aligned bases; and enough 128² tiles
// (>= 64 over the batch) to fill the chip — the IMU encoder's few-tile GEMMs stay on the VALU kernel.
static bool f32_mfma_ok(int M, int N, int K, int batch, const void* A, long sam, long sak, long sAb, const void* B,
                        long sbk, long sbn, long sBb) {
  if (!cmhar_f32_mfma()) return false;
  if ((long)cdiv(M, 128) * cdiv(N, 128) * batch < 64) return false;
  if (!al16(A) || !al16(B) || (sAb & 3) || (sBb & 3)) return false;
  const bool akc = sak == 1, bkc = sbk == 1;
  if (!(akc || sam == 1) || !(bkc || sbn == 1)) return false;
  const long a_ld = akc ? sam : sak, b_ld = bkc ? sbn : sbk;
  if ((a_ld & 3) || (b_ld & 3)) return false;
  if ((akc && (K & 3)) || (!akc && (M & 3)) || (bkc && (K & 3)) || (!bkc && (N & 3))) return false;
  return true;
}

template <typename TO>
static void launch_f32_mfma(int batch, hipStream_t stream, int M, int N, int K, const float* A, long sam, long sak,
                            long sAb, const float* B, long sbk, long sbn, long sBb, TO* C, long ldc, long sCb,
                            const Epilogue& e) {
  const bool akc = sak == 1, bkc = sbk == 1;
  const long a_ld = akc ? sam : sak, b_ld = bkc ? sbn : sbk;
  const dim3 grid(cdiv(M, 64 * FWM) * cdiv(N, 64 * FWN), 1, batch);
  const int nt = 64 * FWM * FWN;
#define FL(AK, BK)                                                                                               \
  gemm_f32_mfma_kernel<FWM, FWN, AK, BK, TO><<<grid, nt, 0, stream>>>(M, N, K, A, a_ld, sAb, B, b_ld, sBb, C, ldc,  \
                                                                      sCb, e)
  if (akc && bkc) FL(true, true);
  else if (akc) FL(true, false);
  else if (bkc) FL(false, true);
  else FL(false, false);
#undef FL
}

// Skinny GEMMs (a handful of 64x64 output tiles over a long K: the video projection / projection heads at M = batch
// rows, K = 768) are bound by the latency of their K loop on a few CUs.  Split K over `splits` batched slices into
// fp32 partials (ws: splits*M*N floats), then combine with the epilogue.
extern "C" int cmhar_gemm_generic_splitk(int in_dtype, int out_dtype, int M, int N, int K, int splits, const void* A,
                                         long sam, long sak, const void* B, long sbk, long sbn, void* C, long ldc,
                                         const Epilogue* epi, float* ws, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (splits < 1 || !ws || in_dtype != out_dtype && !(in_dtype == CMHAR_BF16 && out_dtype == CMHAR_F32)) return -1;
  Epilogue e{};
  e.alpha = 1.f;
  if (epi) e = *epi;
  if (e.rowsum) return -3;
  const int klen = cdiv(cdiv(K, splits), TK) * TK;
  const int S = cdiv(K, klen);
  Epilogue plain{};
  plain.alpha = 1.f;
  // slice s: A advanced by s*klen along k, B likewise; the last slice's K is clamped by running it separately
  const int full = K / klen;                           // slices of exactly klen
  // every slice on one kernel (both give the k-ordered chain per slice, so the choice never changes a bit)
  const bool mf = in_dtype == CMHAR_F32 && f32_mfma_ok(M, N, klen, S, A, sam, sak, (long)klen * sak, B, sbk, sbn,
                                                       (long)klen * sbk);
  dim3 grid(cdiv(N, TN), cdiv(M, TM), full);
#define LAUNCH(TI, GRID, KK, AOFF, BOFF, POFF)                                                                  \
  do {                                                                                                          \
    if (mf)                                                                                                     \
      launch_f32_mfma<float>(GRID.z, stream, M, N, KK, (const float*)A + (AOFF), sam, sak, (long)klen * sak,   \
                             (const float*)B + (BOFF), sbk, sbn, (long)klen * sbk, ws + (POFF), N,             \
                             (long)M * N, plain);                                                               \
    else                                                                                                        \
      gemm_generic_kernel<TI, float><<<GRID, 256, 0, stream>>>(M, N, KK, (const TI*)A + (AOFF), sam, sak,       \
                                                               (long)klen * sak, (const TI*)B + (BOFF), sbk,    \
                                                               sbn, (long)klen * sbk, ws + (POFF), N,           \
                                                               (long)M * N, plain);                             \
  } while (0)
  if (full > 0) {
    if (in_dtype == CMHAR_F32) LAUNCH(float, grid, klen, 0, 0, 0);
    else LAUNCH(bf16, grid, klen, 0, 0, 0);
  }
  if (full < S) {
    const long k0 = (long)full * klen;
    dim3 g1(cdiv(N, TN), cdiv(M, TM), 1);
    if (in_dtype == CMHAR_F32) LAUNCH(float, g1, (int)(K - k0), k0 * sak, k0 * sbk, (long)full * M * N);
    else LAUNCH(bf16, g1, (int)(K - k0), k0 * sak, k0 * sbk, (long)full * M * N);
  }
#undef LAUNCH
  const int blocks = min(1024, cdiv((long)M * N, 256));
  if (out_dtype == CMHAR_F32) generic_splitk_reduce<float><<<blocks, 256, 0, stream>>>(M, N, S, ws, (float*)C, ldc, e);
  else generic_splitk_reduce<bf16><<<blocks, 256, 0, stream>>>(M, N, S, ws, (bf16*)C, ldc, e);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_gemm_generic(int in_dtype, int out_dtype, int M, int N, int K, int batch, const void* A,
                                  long sam, long sak, long sAb, const void* B, long sbk, long sbn, long sBb, void* C,
                                  long ldc, long sCb, const Epilogue* epi, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  Epilogue e{};
  e.alpha = 1.f;
  if (epi) e = *epi;                                   // NULL = the plain product
  if (e.rowsum) return -3;                             // row sums: 256-tile bf16 weight-gradient path only
  // few 64² tiles (the IMU encoder's token GEMMs: M = 13·batch): 32² tiles for 4x the workgroups
  const bool small = (long)cdiv(N, TN) * cdiv(M, TM) * batch < 128;
  dim3 grid(cdiv(N, TN), cdiv(M, TM), batch), grid32(cdiv(N, 32), cdiv(M, 32), batch);
#define LAUNCH(TI, TO)                                                                                          \
  do {                                                                                                          \
    if (small && K >= CMHAR_SMALL_KT)                                                                           \
      gemm_generic_kernel<TI, TO, 32, CMHAR_SMALL_KT><<<grid32, 256, 0, stream>>>(M, N, K, (const TI*)A, sam, sak, sAb, \
                                                                       (const TI*)B, sbk, sbn, sBb, (TO*)C, ldc, sCb, e); \
    else if (small)                                                                                             \
      gemm_generic_kernel<TI, TO, 32><<<grid32, 256, 0, stream>>>(M, N, K, (const TI*)A, sam, sak, sAb,        \
                                                                  (const TI*)B, sbk, sbn, sBb, (TO*)C, ldc, sCb, e); \
    else                                                                                                        \
      gemm_generic_kernel<TI, TO><<<grid, 256, 0, stream>>>(M, N, K, (const TI*)A, sam, sak, sAb, (const TI*)B, \
                                                            sbk, sbn, sBb, (TO*)C, ldc, sCb, e);                \
  } while (0)
  if (in_dtype == CMHAR_F32 && f32_mfma_ok(M, N, K, batch, A, sam, sak, sAb, B, sbk, sbn, sBb) &&
      (out_dtype == CMHAR_F32 || out_dtype == CMHAR_BF16)) {
    if (out_dtype == CMHAR_F32)
      launch_f32_mfma<float>(batch, stream, M, N, K, (const float*)A, sam, sak, sAb, (const float*)B, sbk, sbn, sBb,
                             (float*)C, ldc, sCb, e);
    else
      launch_f32_mfma<bf16>(batch, stream, M, N, K, (const float*)A, sam, sak, sAb, (const float*)B, sbk, sbn, sBb,
                            (bf16*)C, ldc, sCb, e);
  } else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_F32) LAUNCH(float, float);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_BF16) LAUNCH(bf16, bf16);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_F32) LAUNCH(bf16, float);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_BF16) LAUNCH(float, bf16);
  else return -1;
#undef LAUNCH
  CMHAR_CHECK_LAUNCH();
  return 0;
}
