// Row/column normalisations and reductions on the pretraining path.
//   LayerNorm fwd/bwd  — VideoMAE layernorm_before/after (eps 1e-12, modeling_videomae.py:326-358) and the IMU
//                        post-LN `norm1/norm2` (x = LN(res + dropout(sub)), torch transformer.py) + final `norm`.
//                        One wave per row, fp32 statistics, dgamma/dbeta as per-block partial slabs.
//   BatchNorm1d+ReLU   — ProjectionHead / IMUClassifier `Linear → BN → ReLU` (models.py:221-234, 311-322).
//   L2 normalise       — F.normalize(dim=1, eps=1e-12) (models.py:288-289).
//   column sums        — bias gradients and slab reductions.
#include "common.h"

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float elem_drop(unsigned long long seed, float p, long row, int col) {
  return drop_mask(seed, p, row, col);
}

constexpr int MAXPER = 16;   // columns per lane: N <= 1024

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
  float v[MAXPER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < N) {
      float x = to_f<T>(a[row * lda + c]);
      if (b) x += to_f<T>(b[row * ldb + c]) * elem_drop(seed, pdrop, row, c);
      v[i] = x;
      s += x;
    }
  }
  const float mu = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int c = lane + 64 * i;
    if (c < N) { const float d = v[i] - mu; q += d * d; }
  }
  const float r = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int c = lane + 64 * i;
    if (c < N) {
      if (h_out) h_out[row * ldh + c] = from_f<T>(v[i]);
      y[row * ldy + c] = from_f<T>((v[i] - mu) * r * gamma[c] + beta[c]);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = r; }
}

// dh = LN_bwd(dy) (+ dres); db_out (optional) = dh * dropmask(b); dgamma/dbeta partial slabs per block.
// Each block: 4 waves x ROWS_PER_WAVE rows.
constexpr int LN_BWD_ROWS = 16;
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int M, int N, const T* __restrict__ dy, long lddy,
                                                     const T* __restrict__ h, long ldh, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, long ldres, T* __restrict__ dh,
                                                     long lddh, T* __restrict__ db_out, long lddb, float pdrop,
                                                     unsigned long long seed, float* __restrict__ pgamma,
                                                     float* __restrict__ pbeta) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[MAXPER], ab[MAXPER];
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) { ag[i] = 0.f; ab[i] = 0.f; }
  for (int rr = 0; rr < LN_BWD_ROWS; ++rr) {
    const long row = ((long)blockIdx.x * 4 + wave) * LN_BWD_ROWS + rr;
    if (row >= M) break;
    const float mu = mean[row], r = rstd[row];
    float xh[MAXPER], g[MAXPER];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int c = lane + 64 * i;
      xh[i] = 0.f;
      g[i] = 0.f;
      if (c < N) {
        const float d = to_f<T>(dy[row * lddy + c]);
        xh[i] = (to_f<T>(h[row * ldh + c]) - mu) * r;
        g[i] = d * gamma[c];
        ag[i] += d * xh[i];
        ab[i] += d;
        s1 += g[i];
        s2 += g[i] * xh[i];
      }
    }
    s1 = wave_sum(s1) / N;
    s2 = wave_sum(s2) / N;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int c = lane + 64 * i;
      if (c < N) {
        float v = r * (g[i] - s1 - xh[i] * s2);
        if (dres) v += to_f<T>(dres[row * ldres + c]);
        dh[row * lddh + c] = from_f<T>(v);
        if (db_out) db_out[row * lddb + c] = from_f<T>(v * elem_drop(seed, pdrop, row, c));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int c = lane + 64 * i;
    if (c < N) { red[0][wave][c] = ag[i]; red[1][wave][c] = ab[i]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    pgamma[(long)blockIdx.x * N + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pbeta[(long)blockIdx.x * N + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// out[n] = alpha * Σ_m X[m*ldx + n] + beta * out[n]   (fp32 out); two-level: blocks of 64 columns x row chunks.
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(int M, int N, const T* __restrict__ X, long ldx,
                                                             int rows_per_chunk, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * rows_per_chunk;
  const long r1 = min((long)M, r0 + rows_per_chunk);
  float s = 0.f;
  if (col < N)
    for (long r = r0 + sub; r < r1; r += 4) s += to_f<T>(X[r * ldx + col]);
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && col < N) part[(long)blockIdx.y * N + col] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void colsum_final_kernel(int chunks, int N, const float* __restrict__ part, float* __restrict__ out,
                                    float alpha, float beta) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(long)c * N + col];
  out[col] = alpha * s + (beta != 0.f ? beta * out[col] : 0.f);
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
  if (training) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += x[(long)b * C + c];
    mu = s / B;
    float q = 0.f;
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
  for (int b = 0; b < B; ++b) {
    float v = (x[(long)b * C + c] - mu) * r * w[c] + bias[c];
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
  for (int b = 0; b < B; ++b) {
    float g = dy[(long)b * C + c];
    if (relu && y[(long)b * C + c] <= 0.f) g = 0.f;
    const float xh = (x[(long)b * C + c] - mu) * r;
    sg += g;
    sgx += g * xh;
  }
  dw[c] = sgx + (beta != 0.f ? beta * dw[c] : 0.f);
  db[c] = sg + (beta != 0.f ? beta * db[c] : 0.f);
  for (int b = 0; b < B; ++b) {
    float g = dy[(long)b * C + c];
    if (relu && y[(long)b * C + c] <= 0.f) g = 0.f;
    const float xh = (x[(long)b * C + c] - mu) * r;
    dx[(long)b * C + c] = training ? w[c] * r * (g - sg / B - xh * sgx / B) : w[c] * r * g;
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
  if (dtype == CMHAR_BF16)
    ln_fwd_kernel<bf16><<<grid, 256, 0, st>>>(M, N, (const bf16*)a, lda, (const bf16*)b, ldb, pdrop, seed,
                                              (bf16*)h_out, ldh, (bf16*)y, ldy, gamma, beta, mean, rstd, eps);
  else
    ln_fwd_kernel<float><<<grid, 256, 0, st>>>(M, N, (const float*)a, lda, (const float*)b, ldb, pdrop, seed,
                                               (float*)h_out, ldh, (float*)y, ldy, gamma, beta, mean, rstd, eps);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Number of fp32 floats the caller must provide in `ws` for cmhar_layernorm_bwd.
extern "C" long cmhar_layernorm_bwd_ws(int M, int N) { return 2L * cdiv(M, 4 * LN_BWD_ROWS) * N; }

extern "C" int cmhar_colsum(int dtype, int M, int N, const void* X, long ldx, float* out, float alpha, float beta,
                            float* ws, long ws_floats, hipStream_t st);

// dgamma/dbeta are written as out = Σ + beta_acc * out (beta_acc = 1 to accumulate into existing grads).
extern "C" int cmhar_layernorm_bwd(int dtype, int M, int N, const void* dy, long lddy, const void* h, long ldh,
                                   const float* gamma, const float* mean, const float* rstd, const void* dres,
                                   long ldres, void* dh, long lddh, void* db_out, long lddb, float pdrop,
                                   unsigned long long seed, float* dgamma, float* dbeta, float beta_acc, float* ws,
                                   hipStream_t st) {
  if (M <= 0) return 0;
  if (N > 64 * MAXPER) return -1;
  const int blocks = cdiv(M, 4 * LN_BWD_ROWS);
  float* pg = ws;
  float* pb = ws + (long)blocks * N;
  if (dtype == CMHAR_BF16)
    ln_bwd_kernel<bf16><<<blocks, 256, 0, st>>>(M, N, (const bf16*)dy, lddy, (const bf16*)h, ldh, gamma, mean, rstd,
                                                (const bf16*)dres, ldres, (bf16*)dh, lddh, (bf16*)db_out, lddb, pdrop,
                                                seed, pg, pb);
  else
    ln_bwd_kernel<float><<<blocks, 256, 0, st>>>(M, N, (const float*)dy, lddy, (const float*)h, ldh, gamma, mean,
                                                 rstd, (const float*)dres, ldres, (float*)dh, lddh, (float*)db_out,
                                                 lddb, pdrop, seed, pg, pb);
  CMHAR_CHECK_LAUNCH();
  const int g = cdiv(N, 256);
  colsum_final_kernel<<<g, 256, 0, st>>>(blocks, N, pg, dgamma, 1.f, beta_acc);
  colsum_final_kernel<<<g, 256, 0, st>>>(blocks, N, pb, dbeta, 1.f, beta_acc);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" long cmhar_colsum_ws(int M, int N) {
  const int rows_per_chunk = 256;
  return (long)cdiv(M, rows_per_chunk) * N;
}

extern "C" int cmhar_colsum(int dtype, int M, int N, const void* X, long ldx, float* out, float alpha, float beta,
                            float* ws, long ws_floats, hipStream_t st) {
  if (N <= 0) return 0;
  const int rows_per_chunk = 256;
  const int chunks = cdiv(M, rows_per_chunk);
  if ((long)chunks * N > ws_floats) return -2;
  dim3 grid(cdiv(N, 64), chunks);
  if (M > 0) {
    if (dtype == CMHAR_BF16)
      colsum_partial_kernel<bf16><<<grid, 256, 0, st>>>(M, N, (const bf16*)X, ldx, rows_per_chunk, ws);
    else
      colsum_partial_kernel<float><<<grid, 256, 0, st>>>(M, N, (const float*)X, ldx, rows_per_chunk, ws);
  }
  colsum_final_kernel<<<cdiv(N, 256), 256, 0, st>>>(M > 0 ? chunks : 0, N, ws, out, alpha, beta);
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
