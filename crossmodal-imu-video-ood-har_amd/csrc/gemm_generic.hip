// Generic strided GEMM with fp32 accumulation (VALU FMA, LDS-tiled).
//
// Used for (a) the exact-fp32 parity mode of every Linear on the path and (b) the small, latency-bound
// GEMMs of the IMU encoder / projection heads (M = batch*13 or batch rows), where an MFMA tile would idle.
// C[m,n] = epilogue( sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] ), batched over blockIdx.z.
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, TK = 32, NTH = 256;   // default tile; T = 32 for grids of few 64² tiles

// The GEMMs this kernel serves are small (tens of blocks) with K up to a few thousand, so a K-step is bounded by
// memory LATENCY, not bandwidth: tile k+1 is loaded into registers while tile k is consumed from LDS (double-
// buffered LDS, one barrier per K-step), so each step pays compute + one overlapped fetch.
template <typename TIn, int T>
struct GenStage {
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
template <typename TIn, typename TOut, int T = TM>
__global__ __launch_bounds__(NTH) void gemm_generic_kernel(
    int M, int N, int K, const TIn* __restrict__ A, long sam, long sak, long sAb, const TIn* __restrict__ B,
    long sbk, long sbn, long sBb, TOut* __restrict__ C, long ldc, long sCb, Epilogue e) {
  constexpr int R = T / 16;
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
  GenStage<TIn, T> st;
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
  const int esz = in_dtype == CMHAR_BF16 ? 2 : 4;
  // slice s: A advanced by s*klen along k, B likewise; the last slice's K is clamped by running it separately
  const int full = K / klen;                           // slices of exactly klen
  dim3 grid(cdiv(N, TN), cdiv(M, TM), full);
#define LAUNCH(TI, GRID, KK, AOFF, BOFF, POFF)                                                                  \
  gemm_generic_kernel<TI, float><<<GRID, 256, 0, stream>>>(M, N, KK, (const TI*)A + (AOFF), sam, sak,           \
                                                           (long)klen * sak, (const TI*)B + (BOFF), sbk, sbn,   \
                                                           (long)klen * sbk, ws + (POFF), N, (long)M * N, plain)
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
  (void)esz;
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
    if (small)                                                                                                  \
      gemm_generic_kernel<TI, TO, 32><<<grid32, 256, 0, stream>>>(M, N, K, (const TI*)A, sam, sak, sAb,        \
                                                                  (const TI*)B, sbk, sbn, sBb, (TO*)C, ldc, sCb, e); \
    else                                                                                                        \
      gemm_generic_kernel<TI, TO><<<grid, 256, 0, stream>>>(M, N, K, (const TI*)A, sam, sak, sAb, (const TI*)B, \
                                                            sbk, sbn, sBb, (TO*)C, ldc, sCb, e);                \
  } while (0)
  if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_F32) LAUNCH(float, float);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_BF16) LAUNCH(bf16, bf16);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_F32) LAUNCH(bf16, float);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_BF16) LAUNCH(float, bf16);
  else return -1;
#undef LAUNCH
  CMHAR_CHECK_LAUNCH();
  return 0;
}
