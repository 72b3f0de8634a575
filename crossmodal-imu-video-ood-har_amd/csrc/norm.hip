// Row/column normalisations and reductions on the pretraining path.
//   LayerNorm fwd/bwd  — VideoMAE layernorm_before/after (eps 1e-12, modeling_videomae.py:326-358) and the IMU
//                        post-LN `norm1/norm2` (x = LN(res + dropout(sub)), torch transformer.py) + final `norm`.
//                        One wave per row, fp32 statistics, dgamma/dbeta as per-block partial slabs.
//   BatchNorm1d+ReLU   — ProjectionHead / IMUClassifier `Linear → BN → ReLU` (models.py:221-234, 311-322).
//   L2 normalise       — F.normalize(dim=1, eps=1e-12) (models.py:288-289).
//   column sums        — bias gradients and slab reductions.
#include "common.h"
#include "rowops.h"
#include <algorithm>

namespace {

// Two independent wave sums with their shuffle chains interleaved (half the dependent latency of two calls).
__device__ __forceinline__ void wave_sum2(float& a, float& b) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ta = __shfl_xor(a, o), tb = __shfl_xor(b, o);
    a += ta;
    b += tb;
  }
}

__device__ __forceinline__ float elem_drop(unsigned long long seed, float p, long row, int col) {
  return drop_mask(seed, p, row, col);
}

constexpr int MAXPER = 16;   // columns per lane: N <= 1024

// the vectorised LayerNorm kernels need N a multiple of 256 and 4-element aligned leading dimensions
static bool ln_vec_ok(int N, long a, long b, long c) {
  return N % 256 == 0 && N <= 1024 && (a % 4) == 0 && (b % 4) == 0 && (c % 4) == 0;
}

// y = LN(a + drop(b)) with gamma/beta; h_out (optional) = a + drop(b); mean/rstd per row.
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int M, int N, const T* __restrict__ a, long lda,
                                                     const T* __restrict__ b, long ldb, float pdrop,
                                                     unsigned long long seed, T* __restrict__ h_out, long ldh,
                                                     T* __restrict__ y, long ldy, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float* __restrict__ mean,
                                                     float* __restrict__ rstd, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float mu, r;
  ln_row_fwd<T>(lane, row, N, a + row * lda, b ? b + row * ldb : nullptr, pdrop, seed, h_out ? h_out + row * ldh : nullptr,
                y + row * ldy, gamma, beta, eps, mu, r);
  if (lane == 0) { mean[row] = mu; rstd[row] = r; }
}

// Vectorised forward for N % 256 == 0 without the add/dropout input: one wave per row, 4 consecutive columns per
// lane per 256-column group (8-B bf16 / 16-B fp32 accesses), two-pass statistics in registers.  Rows grid-strided
// over LNF_WAVES-wave blocks with the next row's loads issued under the current row's math (one short-lived wave
// per row left the loads of a single row in flight per wave); γ / β loaded once per lane.  Per-row arithmetic as
// before: the same bits.
constexpr int LNF_WAVES = 8;
template <typename T, int G>
__global__ __launch_bounds__(64 * LNF_WAVES) void ln_fwd_vec_kernel(int M, const T* __restrict__ a, long lda,
                                                                    T* __restrict__ y, long ldy,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta,
                                                                    float* __restrict__ mean, float* __restrict__ rstd,
                                                                    float eps) {
  constexpr int N = 256 * G;
  typedef __attribute__((ext_vector_type(4))) T vec4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm[G][4], bt[G][4];
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { gm[i][j] = gamma[256 * i + 4 * lane + j]; bt[i][j] = beta[256 * i + 4 * lane + j]; }
  const long wstride = (long)gridDim.x * LNF_WAVES;
  const long row0 = (long)blockIdx.x * LNF_WAVES + wave;
  vec4 vx[G];
  auto load = [&](long row) {
#pragma unroll
    for (int i = 0; i < G; ++i) vx[i] = *(const vec4*)(a + row * lda + 256 * i + 4 * lane);
  };
  if (row0 < M) load(row0);
  for (long row = row0; row < M; row += wstride) {
    float v[G][4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[i][j] = to_f<T>(vx[i][j]); s += v[i][j]; }
    if (row + wstride < M) load(row + wstride);     // prefetch the next row under this row's math
    const float mu = wave_sum(s) * (1.f / N);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[i][j] - mu; q += d * d; }
    const float r = rsqrtf(wave_sum(q) * (1.f / N) + eps);
#pragma unroll
    for (int i = 0; i < G; ++i) {
      vec4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<T>((v[i][j] - mu) * r * gm[i][j] + bt[i][j]);
      *(vec4*)(y + row * ldy + 256 * i + 4 * lane) = o;
    }
    if (lane == 0) { mean[row] = mu; rstd[row] = r; }
  }
}

// dh = LN_bwd(dy) (+ dres); db_out (optional) = dh * dropmask(b); dgamma/dbeta partial slabs per block.
// Each block: 4 waves x ROWS_PER_WAVE rows.
constexpr int LN_BWD_ROWS = 16;
template <typename T, int MP = MAXPER>   // MP: columns per lane (N <= 64·MP)
__global__ __launch_bounds__(256) void ln_bwd_kernel(int M, int N, const T* __restrict__ dy, long lddy,
                                                     const T* __restrict__ h, long ldh, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, long ldres, T* __restrict__ dh,
                                                     long lddh, T* __restrict__ db_out, long lddb, float pdrop,
                                                     unsigned long long seed, float* __restrict__ pgamma,
                                                     float* __restrict__ pbeta) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[MP], ab[MP];
#pragma unroll
  for (int i = 0; i < MP; ++i) { ag[i] = 0.f; ab[i] = 0.f; }
  // rows in groups of LN_BWD_PF whose dy / h / statistics loads are all issued before the first row's reductions
  // (one row at a time, each row's loads waited on the previous row's cross-lane sums: the M = 416 IMU LayerNorms
  // ran ~16 exposed load latencies per wave); per-row arithmetic and accumulation order unchanged
  constexpr int LN_BWD_PF = 4;
  const long row0 = ((long)blockIdx.x * 4 + wave) * LN_BWD_ROWS;
  for (int rg = 0; rg < LN_BWD_ROWS; rg += LN_BWD_PF) {
    if (row0 + rg >= M) break;
    float pd[LN_BWD_PF][MP], ph[LN_BWD_PF][MP], pmu[LN_BWD_PF], prs[LN_BWD_PF];
#pragma unroll
    for (int u = 0; u < LN_BWD_PF; ++u) {
      const long row = row0 + rg + u;
      const bool ok = row < M;
      pmu[u] = ok ? mean[row] : 0.f;
      prs[u] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < MP; ++i) {
        const int c = lane + 64 * i;
        pd[u][i] = ok && c < N ? to_f<T>(dy[row * lddy + c]) : 0.f;
        ph[u][i] = ok && c < N ? to_f<T>(h[row * ldh + c]) : 0.f;
      }
    }
#pragma unroll
  for (int u = 0; u < LN_BWD_PF; ++u) {
    const long row = row0 + rg + u;
    if (row >= M) break;
    float gx[MP];
    ln_row_bwd<MP>(lane, N, pd[u], ph[u], pmu[u], prs[u], gamma, ag, ab, gx);
#pragma unroll
    for (int i = 0; i < MP; ++i) {
      const int c = lane + 64 * i;
      if (c < N) {
        float v = gx[i];
        if (dres) v += to_f<T>(dres[row * ldres + c]);
        dh[row * lddh + c] = from_f<T>(v);
        if (db_out) db_out[row * lddb + c] = from_f<T>(v * elem_drop(seed, pdrop, row, c));
      }
    }
  }
  }
#pragma unroll
  for (int i = 0; i < MP; ++i) {
    const int c = lane + 64 * i;
    if (c < N) { red[0][wave][c] = ag[i]; red[1][wave][c] = ab[i]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    pgamma[(long)blockIdx.x * 2 * N + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pbeta[(long)blockIdx.x * 2 * N + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// out[n] = alpha * Σ_m X[m*ldx + n] + beta * out[n]   (fp32 out).  Two levels, both parallel over rows:
//   partial: block = 4 waves x (64 lanes x 4 consecutive columns) over a chunk of rows → part[chunk][N]
//   final:   block = 4 row-groups x 64 columns over all chunks, LDS tree → out
constexpr int CS_VEC = 4;
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(int M, int N, const T* __restrict__ X, long ldx,
                                                             int rows_per_chunk, float* __restrict__ part) {
  __shared__ float red[4][64 * CS_VEC];
  const int lane = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 64 * CS_VEC + lane * CS_VEC;
  const long r0 = (long)blockIdx.y * rows_per_chunk;
  const long r1 = min((long)M, r0 + rows_per_chunk);
  float s[CS_VEC] = {0.f, 0.f, 0.f, 0.f};
  const bool vec = (c0 + CS_VEC <= N) && ((ldx & 3) == 0) && (((uintptr_t)X & 15) == 0);
  if (vec) {
    for (long r = r0 + sub; r < r1; r += 4) {
      const T* p = X + r * ldx + c0;
      if constexpr (sizeof(T) == 2) {
        const bf16x4 v = *(const bf16x4*)p;
#pragma unroll
        for (int j = 0; j < CS_VEC; ++j) s[j] += (float)v[j];
      } else {
        const floatx4 v = *(const floatx4*)p;
#pragma unroll
        for (int j = 0; j < CS_VEC; ++j) s[j] += v[j];
      }
    }
  } else {
    for (long r = r0 + sub; r < r1; r += 4)
#pragma unroll
      for (int j = 0; j < CS_VEC; ++j)
        if (c0 + j < N) s[j] += to_f<T>(X[r * ldx + c0 + j]);
  }
#pragma unroll
  for (int j = 0; j < CS_VEC; ++j) red[sub][lane * CS_VEC + j] = s[j];
  __syncthreads();
  const int t = threadIdx.x;
  const int col = blockIdx.x * 64 * CS_VEC + t;
  if (col < N) part[(long)blockIdx.y * N + col] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

__global__ __launch_bounds__(256) void colsum_final_kernel(int chunks, int N, const float* __restrict__ part,
                                                           float* __restrict__ out, float alpha, float beta) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < N)
    for (int c = g; c < chunks; c += 4) s += part[(long)c * N + col];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    out[col] = alpha * t + (beta != 0.f ? beta * out[col] : 0.f);
  }
}

// As colsum_final_kernel over [chunks][2*N2] partials whose columns [0, N2) go to out0 and [N2, 2*N2) to out1
// (the interleaved dγ | dβ partial rows of the LayerNorm backward: one launch reduces both).
__global__ __launch_bounds__(256) void colsum_final2_kernel(int chunks, int N2, const float* __restrict__ part,
                                                            float* __restrict__ out0, float* __restrict__ out1,
                                                            float beta) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int N = 2 * N2;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < N)
    for (int c = g; c < chunks; c += 4) s += part[(long)c * N + col];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    float* o = col < N2 ? out0 + col : out1 + (col - N2);
    *o = t + (beta != 0.f ? beta * *o : 0.f);
  }
}

// One-launch form of colsum_partial + colsum_final2 for up to RR1_MAX partial rows (the LayerNorm backward's 512
// per-block rows): 16 columns × 16 row slots per block, each slot summing its rows with 8 independent partial sums
// (8 loads in flight), then the 16 slots combined through LDS — fixed order throughout.  (The two launches of ~5 µs
// each were mostly launch and dependent-load latency.)
constexpr int RR1_MAX = 1024;
__global__ __launch_bounds__(256) void colsum_rows2_kernel(int rows, int N2, const float* __restrict__ part,
                                                           float* __restrict__ out0, float* __restrict__ out1,
                                                           float beta) {
  __shared__ float red[16][17];
  const int N = 2 * N2;
  const int cl = threadIdx.x & 15, slot = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    int r = slot;
    for (; r + 7 * 16 < rows; r += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += part[(long)(r + 16 * u) * N + col];
    }
    for (; r < rows; r += 16) a[0] += part[(long)r * N + col];
  }
  red[slot][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (slot == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    float* o = col < N2 ? out0 + col : out1 + (col - N2);
    *o = t + (beta != 0.f ? beta * *o : 0.f);
  }
}

// BatchNorm1d (+ optional ReLU) over x [B][C] fp32: one thread per channel.
__global__ void bn_fwd_kernel(int B, int C, const float* __restrict__ x, float* __restrict__ y,
                              const float* __restrict__ w, const float* __restrict__ bias,
                              float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ smean,
                              float* __restrict__ srstd, int training, float momentum, float eps, int relu,
                              long long* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mu, r;
  if (training && nbt && c == 0) *nbt += 1;   // num_batches_tracked
  // (the b loops unrolled: their loads issue together instead of one dependent-latency round trip per row — one
  // thread per channel, a few hundred threads in all; the summation order is unchanged)
  if (training) {
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < B; ++b) s += x[(long)b * C + c];
    mu = s / B;
    float q = 0.f;
#pragma unroll 8
    for (int b = 0; b < B; ++b) { const float d = x[(long)b * C + c] - mu; q += d * d; }
    const float var = q / B;
    r = rsqrtf(var + eps);
    if (rmean) {
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * B / (B - 1);
    }
  } else {
    mu = rmean[c];
    r = rsqrtf(rvar[c] + eps);
  }
  smean[c] = mu;
  srstd[c] = r;
  const float wc = w[c], bc = bias[c];
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    float v = (x[(long)b * C + c] - mu) * r * wc + bc;
    if (relu) v = fmaxf(v, 0.f);
    y[(long)b * C + c] = v;
  }
}

// Backward of y = relu?(BN(x)): needs x, saved mean/rstd, y (for the relu mask).
__global__ void bn_bwd_kernel(int B, int C, const float* __restrict__ x, const float* __restrict__ y,
                              const float* __restrict__ dy, const float* __restrict__ w,
                              const float* __restrict__ smean, const float* __restrict__ srstd, float* __restrict__ dx,
                              float* __restrict__ dw, float* __restrict__ db, int training, int relu, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mu = smean[c], r = srstd[c];
  float sg = 0.f, sgx = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    float g = dy[(long)b * C + c];
    if (relu && y[(long)b * C + c] <= 0.f) g = 0.f;
    const float xh = (x[(long)b * C + c] - mu) * r;
    sg += g;
    sgx += g * xh;
  }
  dw[c] = sgx + (beta != 0.f ? beta * dw[c] : 0.f);
  db[c] = sg + (beta != 0.f ? beta * db[c] : 0.f);
  const float wc = w[c];
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    float g = dy[(long)b * C + c];
    if (relu && y[(long)b * C + c] <= 0.f) g = 0.f;
    const float xh = (x[(long)b * C + c] - mu) * r;
    dx[(long)b * C + c] = training ? wc * r * (g - sg / B - xh * sgx / B) : wc * r * g;
  }
}

// y = x / max(||x||, eps) rowwise; one wave per row.
__global__ void l2n_fwd_kernel(int M, int N, const float* __restrict__ x, float* __restrict__ y,
                               float* __restrict__ norm, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) { const float v = x[row * N + c]; s += v * v; }
  const float n = sqrtf(wave_sum(s));
  const float d = fmaxf(n, eps);
  for (int c = lane; c < N; c += 64) y[row * N + c] = x[row * N + c] / d;
  if (lane == 0) norm[row] = n;
}

__global__ void l2n_bwd_kernel(int M, int N, const float* __restrict__ y, const float* __restrict__ dy,
                               const float* __restrict__ norm, float* __restrict__ dx, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float n = norm[row];
  if (n > eps) {
    float s = 0.f;
    for (int c = lane; c < N; c += 64) s += y[row * N + c] * dy[row * N + c];
    s = wave_sum(s);
    for (int c = lane; c < N; c += 64) dx[row * N + c] = (dy[row * N + c] - y[row * N + c] * s) / n;
  } else {
    for (int c = lane; c < N; c += 64) dx[row * N + c] = dy[row * N + c] / eps;
  }
}

}  // namespace

extern "C" int cmhar_layernorm_fwd(int dtype, int M, int N, const void* a, long lda, const void* b, long ldb,
                                   float pdrop, unsigned long long seed, void* h_out, long ldh, void* y, long ldy,
                                   const float* gamma, const float* beta, float* mean, float* rstd, float eps,
                                   hipStream_t st) {
  if (M <= 0) return 0;
  if (N > 64 * MAXPER) return -1;
  const int grid = cdiv(M, 4);
  if (!b && !h_out && ln_vec_ok(N, lda, ldy, ldy)) {
    // 512-thread blocks, rows grid-strided: three per CU (256 CUs) for N <= 768 (72 VGPRs: 7 waves per SIMD), two
    // above
    const int vgrid = std::min(N <= 768 ? 768 : 512, cdiv(M, LNF_WAVES));
#define LF(TT, G) ln_fwd_vec_kernel<TT, G><<<vgrid, 64 * LNF_WAVES, 0, st>>>(M, (const TT*)a, lda, (TT*)y, ldy, gamma, beta, mean, rstd, eps)
    const int G = N / 256;
    if (dtype == CMHAR_BF16) {
      switch (G) { case 1: LF(bf16, 1); break; case 2: LF(bf16, 2); break; case 3: LF(bf16, 3); break; default: LF(bf16, 4); }
    } else if (dtype == CMHAR_F16) {
      switch (G) { case 1: LF(f16, 1); break; case 2: LF(f16, 2); break; case 3: LF(f16, 3); break; default: LF(f16, 4); }
    } else {
      switch (G) { case 1: LF(float, 1); break; case 2: LF(float, 2); break; case 3: LF(float, 3); break; default: LF(float, 4); }
    }
#undef LF
  } else if (dtype == CMHAR_BF16)
    ln_fwd_kernel<bf16><<<grid, 256, 0, st>>>(M, N, (const bf16*)a, lda, (const bf16*)b, ldb, pdrop, seed,
                                              (bf16*)h_out, ldh, (bf16*)y, ldy, gamma, beta, mean, rstd, eps);
  else if (dtype == CMHAR_F16)
    ln_fwd_kernel<f16><<<grid, 256, 0, st>>>(M, N, (const f16*)a, lda, (const f16*)b, ldb, pdrop, seed,
                                             (f16*)h_out, ldh, (f16*)y, ldy, gamma, beta, mean, rstd, eps);
  else
    ln_fwd_kernel<float><<<grid, 256, 0, st>>>(M, N, (const float*)a, lda, (const float*)b, ldb, pdrop, seed,
                                               (float*)h_out, ldh, (float*)y, ldy, gamma, beta, mean, rstd, eps);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Sum `rows` fp32 partial rows [rows][N] into out (alpha/beta), via a second partial level when rows is large.
// Partial-row reduction of per-block partial sums (a few hundred rows of N or 2N columns): chunks of >= 8 rows, at
// most 64 of them, so the partial pass has ~(N/256)·64 workgroups instead of a handful of long row loops (the LN
// backward's 512 x 1536 partials: 21 -> ~5 us per call).
static int rr_chunks(int rows) { return std::min(64, cdiv(rows, 8)); }
static long reduce_rows_ws(int rows, int N) { return rows > 32 ? (long)rr_chunks(rows) * N : 0; }
static void reduce_rows(const float* part, int rows, int N, float* out, float alpha, float beta, float* scratch,
                        hipStream_t st) {
  if (rows > 32) {
    const int chunks = rr_chunks(rows), rpc = cdiv(rows, chunks);
    colsum_partial_kernel<float><<<dim3(cdiv(N, 64 * CS_VEC), chunks), 256, 0, st>>>(rows, N, part, N, rpc,
                                                                                     scratch);
    colsum_final_kernel<<<cdiv(N, 64), 256, 0, st>>>(chunks, N, scratch, out, alpha, beta);
  } else {
    colsum_final_kernel<<<cdiv(N, 64), 256, 0, st>>>(rows, N, part, out, alpha, beta);
  }
}

// dγ and dβ from interleaved partial rows [rows][dγ(N) | dβ(N)] in one (or two, for many rows) launches.
static void reduce_rows_gb(const float* part, int rows, int N, float* dgamma, float* dbeta, float beta,
                           float* scratch, hipStream_t st) {
  if (rows > 32 && rows <= RR1_MAX) {
    colsum_rows2_kernel<<<cdiv(2 * N, 16), 256, 0, st>>>(rows, N, part, dgamma, dbeta, beta);
  } else if (rows > 32) {
    const int chunks = rr_chunks(rows), rpc = cdiv(rows, chunks);
    colsum_partial_kernel<float><<<dim3(cdiv(2 * N, 64 * CS_VEC), chunks), 256, 0, st>>>(rows, 2 * N, part, 2 * N,
                                                                                         rpc, scratch);
    colsum_final2_kernel<<<cdiv(2 * N, 64), 256, 0, st>>>(chunks, N, scratch, dgamma, dbeta, beta);
  } else {
    colsum_final2_kernel<<<cdiv(2 * N, 64), 256, 0, st>>>(rows, N, part, dgamma, dbeta, beta);
  }
}

// Vectorised LayerNorm backward for N % 256 == 0 (VideoMAE hidden 768): 8 waves per block, rows grid-strided over
// all waves; each lane owns N/256 groups of 4 consecutive columns (8-B bf16 / 16-B fp32 loads), the next row's dy,
// h and residual gradient prefetched into registers under the current row's math.
constexpr int LNV_WAVES = 8;
template <typename T, int G>
__global__ __launch_bounds__(512) void ln_bwd_vec_kernel(int M, const T* __restrict__ dy, long lddy,
                                                         const T* __restrict__ h, long ldh,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         const T* __restrict__ dres, long ldres, T* __restrict__ dh,
                                                         long lddh, float* __restrict__ pgamma,
                                                         float* __restrict__ pbeta) {
  constexpr int N = 256 * G;
  __shared__ float red[2][LNV_WAVES][N];
  typedef __attribute__((ext_vector_type(4))) T vec4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gam[G][4], ag[G][4], ab[G][4];
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { gam[i][j] = gamma[256 * i + 4 * lane + j]; ag[i][j] = 0.f; ab[i][j] = 0.f; }
  // grid-stride over rows: every wave of the (two-per-CU) grid takes rows w, w + W, w + 2W, ...  (W = all waves)
  const long wstride = (long)gridDim.x * LNV_WAVES;
  const long row0 = (long)blockIdx.x * LNV_WAVES + wave;
  vec4 vdy[G], vh[G], vr[G];
  auto load = [&](long row) {   // dy, h and the residual gradient of one row, all issued before any is used
#pragma unroll
    for (int i = 0; i < G; ++i) {
      vdy[i] = *(const vec4*)(dy + row * lddy + 256 * i + 4 * lane);
      vh[i] = *(const vec4*)(h + row * ldh + 256 * i + 4 * lane);
      if (dres) vr[i] = *(const vec4*)(dres + row * ldres + 256 * i + 4 * lane);
    }
  };
  if (row0 < M) load(row0);
  for (long row = row0; row < M; row += wstride) {
    float d[G][4], xh[G][4], rs[G][4];
    const float mu = mean[row], r = rstd[row];
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d[i][j] = to_f<T>(vdy[i][j]);
        xh[i][j] = (to_f<T>(vh[i][j]) - mu) * r;
        rs[i][j] = dres ? to_f<T>(vr[i][j]) : 0.f;
      }
    if (row + wstride < M) load(row + wstride);     // prefetch the next row under this row's math
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g = d[i][j] * gam[i][j];
        ag[i][j] += d[i][j] * xh[i][j];
        ab[i][j] += d[i][j];
        s1 += g;
        s2 += g * xh[i][j];
      }
    wave_sum2(s1, s2);
    s1 *= 1.f / N;
    s2 *= 1.f / N;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      vec4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<T>(r * (d[i][j] * gam[i][j] - s1 - xh[i][j] * s2) + rs[i][j]);
      *(vec4*)(dh + row * lddh + 256 * i + 4 * lane) = o;
    }
  }
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { red[0][wave][256 * i + 4 * lane + j] = ag[i][j]; red[1][wave][256 * i + 4 * lane + j] = ab[i][j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 512) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < LNV_WAVES; ++w) { sg += red[0][w][c]; sb += red[1][w][c]; }
    pgamma[(long)blockIdx.x * 2 * N + c] = sg;
    pbeta[(long)blockIdx.x * 2 * N + c] = sb;
  }
}

static int ln_bwd_blocks(int M, int N, bool vec) {
  // vector path: a balanced grid of at most two 512-thread blocks per CU (256 CUs), rows grid-strided
  return vec ? std::min(512, cdiv(M, LNV_WAVES)) : cdiv(M, 4 * LN_BWD_ROWS);
}

// Number of fp32 floats the caller must provide in `ws` for cmhar_layernorm_bwd (upper bound over both paths).
extern "C" long cmhar_layernorm_bwd_ws(int M, int N) {
  const int blocks = std::max(ln_bwd_blocks(M, N, false), ln_bwd_blocks(M, N, true));
  return 2L * blocks * N + reduce_rows_ws(blocks, 2 * N);
}

// dgamma/dbeta are written as out = Σ + beta_acc * out (beta_acc = 1 to accumulate into existing grads).
extern "C" int cmhar_layernorm_bwd(int dtype, int M, int N, const void* dy, long lddy, const void* h, long ldh,
                                   const float* gamma, const float* mean, const float* rstd, const void* dres,
                                   long ldres, void* dh, long lddh, void* db_out, long lddb, float pdrop,
                                   unsigned long long seed, float* dgamma, float* dbeta, float beta_acc, float* ws,
                                   hipStream_t st) {
  if (M <= 0) return 0;
  if (N > 64 * MAXPER) return -1;
  const bool vec = !db_out && ln_vec_ok(N, lddy, ldh, lddh) && (!dres || ldres % 4 == 0);
  const int blocks = ln_bwd_blocks(M, N, vec);
  float* pg = ws;                                       // partial rows [blocks][dγ | dβ], row stride 2N
  float* pb = ws + N;
  float* scr = ws + 2L * blocks * N;
  if (vec) {
#define LV(TT, G)                                                                                             \
  ln_bwd_vec_kernel<TT, G><<<blocks, 512, 0, st>>>(M, (const TT*)dy, lddy, (const TT*)h, ldh, gamma, mean, rstd, \
                                                   (const TT*)dres, ldres, (TT*)dh, lddh, pg, pb)
    const int G = N / 256;
    if (dtype == CMHAR_BF16) {
      switch (G) { case 1: LV(bf16, 1); break; case 2: LV(bf16, 2); break; case 3: LV(bf16, 3); break; default: LV(bf16, 4); }
    } else {
      switch (G) { case 1: LV(float, 1); break; case 2: LV(float, 2); break; case 3: LV(float, 3); break; default: LV(float, 4); }
    }
#undef LV
  } else if (dtype == CMHAR_BF16) {
    ln_bwd_kernel<bf16><<<blocks, 256, 0, st>>>(M, N, (const bf16*)dy, lddy, (const bf16*)h, ldh, gamma, mean, rstd,
                                                (const bf16*)dres, ldres, (bf16*)dh, lddh, (bf16*)db_out, lddb, pdrop,
                                                seed, pg, pb);
  } else {
    if (N <= 128)   // the IMU encoder / fusion LayerNorms (d = 128): two columns per lane, small prefetch set
      ln_bwd_kernel<float, 2><<<blocks, 256, 0, st>>>(M, N, (const float*)dy, lddy, (const float*)h, ldh, gamma,
                                                      mean, rstd, (const float*)dres, ldres, (float*)dh, lddh,
                                                      (float*)db_out, lddb, pdrop, seed, pg, pb);
    else
      ln_bwd_kernel<float><<<blocks, 256, 0, st>>>(M, N, (const float*)dy, lddy, (const float*)h, ldh, gamma, mean,
                                                   rstd, (const float*)dres, ldres, (float*)dh, lddh, (float*)db_out,
                                                   lddb, pdrop, seed, pg, pb);
  }
  CMHAR_CHECK_LAUNCH();
  reduce_rows_gb(pg, blocks, N, dgamma, dbeta, beta_acc, scr, st);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// rows per partial chunk: 256, or fewer for short columns (the IMU / head bias gradients, M = 13·batch rows) so the
// partial pass still has up to 64 chunks of rows in flight
static int cs_rows(int M) { return M >= 64 * 256 ? 256 : std::max(8, cdiv(M, 64)); }
extern "C" long cmhar_colsum_ws(int M, int N) {
  const int chunks = cdiv(M, cs_rows(M));
  return (long)chunks * N + reduce_rows_ws(chunks, N);
}

extern "C" int cmhar_colsum(int dtype, int M, int N, const void* X, long ldx, float* out, float alpha, float beta,
                            float* ws, long ws_floats, hipStream_t st) {
  if (N <= 0) return 0;
  const int rpc = cs_rows(M), chunks = cdiv(M, rpc);
  if ((long)chunks * N + reduce_rows_ws(chunks, N) > ws_floats) return -2;
  if (M > 0) {
    dim3 grid(cdiv(N, 64 * CS_VEC), chunks);
    if (dtype == CMHAR_BF16)
      colsum_partial_kernel<bf16><<<grid, 256, 0, st>>>(M, N, (const bf16*)X, ldx, rpc, ws);
    else
      colsum_partial_kernel<float><<<grid, 256, 0, st>>>(M, N, (const float*)X, ldx, rpc, ws);
  }
  reduce_rows(ws, M > 0 ? chunks : 0, N, out, alpha, beta, ws + (long)chunks * N, st);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_batchnorm_fwd(int B, int C, const float* x, float* y, const float* w, const float* bias,
                                   float* rmean, float* rvar, float* smean, float* srstd, int training,
                                   float momentum, float eps, int relu, long long* num_batches_tracked,
                                   hipStream_t st) {
  bn_fwd_kernel<<<cdiv(C, 128), 128, 0, st>>>(B, C, x, y, w, bias, rmean, rvar, smean, srstd, training, momentum,
                                              eps, relu, num_batches_tracked);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_batchnorm_bwd(int B, int C, const float* x, const float* y, const float* dy, const float* w,
                                   const float* smean, const float* srstd, float* dx, float* dw, float* db,
                                   int training, int relu, float beta_acc, hipStream_t st) {
  bn_bwd_kernel<<<cdiv(C, 128), 128, 0, st>>>(B, C, x, y, dy, w, smean, srstd, dx, dw, db, training, relu, beta_acc);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_l2normalize_fwd(int M, int N, const float* x, float* y, float* norm, float eps, hipStream_t st) {
  l2n_fwd_kernel<<<cdiv(M, 4), 256, 0, st>>>(M, N, x, y, norm, eps);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_l2normalize_bwd(int M, int N, const float* y, const float* dy, const float* norm, float* dx,
                                     float eps, hipStream_t st) {
  l2n_bwd_kernel<<<cdiv(M, 4), 256, 0, st>>>(M, N, y, dy, norm, dx, eps);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
