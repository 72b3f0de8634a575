// SigmoidContrastiveLoss (src/models/losses.py:25-54), fused forward + analytic backward.
//
//   S_ij = (a_i · b_j) * exp(t) + bias,  labels = 2I - 1,
//   loss = mean_ij BCEWithLogits(z_ij = S_ij*label_ij, y_ij = (label_ij+1)/2)      (= mean softplus(-S))
// computed literally per element so the reference's numerics (max(z,0) - z*y + log1p(exp(-|z|))) are kept.
// a, b are the (globally gathered) unit embeddings [Ba][D], [Bb][D]; gradients are produced for the rows
// [a_off, a_off + a_cnt) of a and [b_off, b_off + b_cnt) of b (the local shard under data parallelism), and for
// t / bias (device scalars; autograd accumulates them — the reference never zeroes them, trainer.py:138).
#include "common.h"

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one block (256 threads) per row i of S: computes S_i·, per-row loss, dS_i· (into ws), da_i, and row partials
__global__ __launch_bounds__(256) void siglip_rows(int Ba, int Bb, int D, const float* __restrict__ a,
                                                   const float* __restrict__ b, const float* __restrict__ t_ptr,
                                                   const float* __restrict__ bias_ptr, float* __restrict__ dS,
                                                   float* __restrict__ row_loss, float* __restrict__ row_dt,
                                                   float* __restrict__ row_db, float* __restrict__ da, int a_off,
                                                   int a_cnt, float inv_n) {
  __shared__ float arow[1024];
  __shared__ float sdS[1024];
  __shared__ float red[3][4];
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float et = __expf(*t_ptr), bias = *bias_ptr;
  for (int k = threadIdx.x; k < D; k += 256) arow[k] = a[(long)i * D + k];
  __syncthreads();
  float l_acc = 0.f, dt_acc = 0.f, db_acc = 0.f;
  for (int j = wave; j < Bb; j += 4) {
    float dot = 0.f;
    for (int k = lane; k < D; k += 64) dot += arow[k] * b[(long)j * D + k];
    dot = wave_sum(dot);
    const float s = dot * et + bias;
    const float lab = (i == j) ? 1.f : -1.f;
    const float z = s * lab, y = (i == j) ? 1.f : 0.f;
    const float l = fmaxf(z, 0.f) - z * y + log1pf(__expf(-fabsf(z)));
    const float sig = 1.f / (1.f + __expf(-z));
    const float ds = (sig - y) * lab * inv_n;         // dloss/dS_ij
    if (lane == 0) {
      sdS[j] = ds;
      dS[(long)i * Bb + j] = ds;
      l_acc += l;
      dt_acc += ds * dot * et;
      db_acc += ds;
    }
  }
  if (lane == 0) { red[0][wave] = l_acc; red[1][wave] = dt_acc; red[2][wave] = db_acc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    row_loss[i] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    row_dt[i] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    row_db[i] = red[2][0] + red[2][1] + red[2][2] + red[2][3];
  }
  if (i >= a_off && i < a_off + a_cnt) {
    for (int k = threadIdx.x; k < D; k += 256) {
      float s = 0.f;
      for (int j = 0; j < Bb; ++j) s += sdS[j] * b[(long)j * D + k];
      da[(long)(i - a_off) * D + k] = s * et;
    }
  }
}

// one block per local column j: db_j = exp(t) Σ_i dS_ij a_i
__global__ __launch_bounds__(256) void siglip_cols(int Ba, int Bb, int D, const float* __restrict__ a,
                                                   const float* __restrict__ t_ptr, const float* __restrict__ dS,
                                                   float* __restrict__ dbv, int b_off) {
  const int j = b_off + blockIdx.x;
  const float et = __expf(*t_ptr);
  for (int k = threadIdx.x; k < D; k += 256) {
    float s = 0.f;
    for (int i = 0; i < Ba; ++i) s += dS[(long)i * Bb + j] * a[(long)i * D + k];
    dbv[(long)blockIdx.x * D + k] = s * et;
  }
}

__global__ void siglip_final(int Ba, const float* __restrict__ row_loss, const float* __restrict__ row_dt,
                             const float* __restrict__ row_db, float inv_n, float* __restrict__ loss,
                             float* __restrict__ gt, float* __restrict__ gbias, float grad_scale) {
  __shared__ float red[3][256];
  float l = 0.f, dt = 0.f, db = 0.f;
  for (int i = threadIdx.x; i < Ba; i += 256) { l += row_loss[i]; dt += row_dt[i]; db += row_db[i]; }
  red[0][threadIdx.x] = l;
  red[1][threadIdx.x] = dt;
  red[2][threadIdx.x] = db;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *loss = red[0][0] * inv_n;
    if (gt) *gt = grad_scale * red[1][0];
    if (gbias) *gbias = grad_scale * red[2][0];
  }
}

}  // namespace

extern "C" long cmhar_siglip_ws(int Ba, int Bb) { return (long)Ba * Bb + 3L * Ba; }

// loss: device fp32 scalar.  da: [a_cnt][D], db: [b_cnt][D] (gradients of the MEAN loss, i.e. dloss/da with
// grad_output = 1; the caller scales by the incoming gradient).  gt / gbias (nullable): dloss/dt, dloss/dbias (overwritten).
extern "C" int cmhar_siglip_loss(int Ba, int Bb, int D, const float* a, const float* b, const float* t,
                                 const float* bias, float* loss, float* da, int a_off, int a_cnt, float* db_vec,
                                 int b_off, int b_cnt, float* gt, float* gbias, float* ws, hipStream_t st) {
  if (D > 1024 || Bb > 1024) return -1;
  const float inv_n = 1.f / ((float)Ba * (float)Bb);
  float* dS = ws;
  float* rl = ws + (long)Ba * Bb;
  float* rdt = rl + Ba;
  float* rdb = rdt + Ba;
  siglip_rows<<<Ba, 256, 0, st>>>(Ba, Bb, D, a, b, t, bias, dS, rl, rdt, rdb, da, a_off, a_cnt, inv_n);
  if (b_cnt > 0) siglip_cols<<<b_cnt, 256, 0, st>>>(Ba, Bb, D, a, t, dS, db_vec, b_off);
  siglip_final<<<1, 256, 0, st>>>(Ba, rl, rdt, rdb, inv_n, loss, gt, gbias, 1.f);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
