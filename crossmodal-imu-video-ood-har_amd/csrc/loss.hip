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

// ---------------------------------------------------------------------------------------------------------------
// Row-softmax cross-entropy family (replaces: nn.CrossEntropyLoss in ClassificationTrainer, trainer.py:249,300;
// FocalLoss losses.py:90-116; LabelSmoothingCrossEntropy losses.py:119-150; the two F.cross_entropy of InfoNCELoss
// losses.py:76-85).  One wave per row of the (strided) logit view z[r][c] = L[r*s_row + c*s_col]:
//   p = softmax(z),  q = (1-eps)·onehot(y) + eps/C,  ce = -Σ q log p,  pt = p_y
//   loss_r = alpha·(1-pt)^gamma·ce        (gamma = 0, alpha = 1: plain / label-smoothed CE)
//   dloss_r/dz = alpha·[(1-pt)^gamma·(p - q) + gamma·(1-pt)^(gamma-1)·pt·ce·(p - onehot)]   (eps = 0 when gamma ≠ 0)
// Rows with y == ignore_index contribute nothing (torch's ignore_index; mean over the others).  labels == NULL:
// y = row index (InfoNCE's arange labels).  Per-row losses and the argmax go to the workspace; a one-block pass
// reduces them in a fixed order (deterministic) and scales the gradients of the mean by 1/count.
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xent_rows(int N, int C, const float* __restrict__ L, long s_row, long s_col,
                                                 const long* __restrict__ labels, long ignore_index, float eps,
                                                 float gamma, float alpha, float* __restrict__ row_loss,
                                                 int* __restrict__ row_state, long* __restrict__ pred) {
  const int row = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;                                   // wave-uniform
  const float* z = L + (long)row * s_row;
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int j = lane; j < C; j += 64) {
    const float v = z[(long)j * s_col];
    if (v > m) { m = v; am = j; }                         // first maximum (torch.argmax's tie rule)
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float mo = __shfl_xor(m, off);
    const int ao = __shfl_xor(am, off);
    if (mo > m || (mo == m && ao < am)) { m = mo; am = ao; }
  }
  float s = 0.f, sz = 0.f;
  for (int j = lane; j < C; j += 64) {
    const float v = z[(long)j * s_col];
    s += __expf(v - m);
    sz += v;
  }
  s = wave_sum(s);
  sz = wave_sum(sz);
  const long y = labels ? labels[row] : (long)row;
  if (lane == 0) {
    if (pred) pred[row] = am;
    int st = 1;
    float l = 0.f;
    if (y == ignore_index) {
      st = 0;
    } else if (y < 0 || y >= C) {
      st = 2;                                             // invalid target: the host raises, like torch
      l = NAN;
    } else {
      const float lse = m + __logf(s);
      const float zy = z[y * s_col];
      const float ce = (1.f - eps) * (lse - zy) + eps * (lse - sz / (float)C);
      if (gamma != 0.f) {
        const float pt = __expf(-ce);
        l = alpha * __powf(fmaxf(1.f - pt, 0.f), gamma) * ce;
      } else {
        l = alpha * ce;
      }
    }
    row_loss[row] = l;
    row_state[row] = st | (am == (int)y ? 4 : 0);
  }
}

// one block: count = #non-ignored rows, loss = Σ row_loss (/count for the mean), correct = #(argmax == y)
__global__ __launch_bounds__(256) void xent_final(int N, const float* __restrict__ row_loss,
                                                  const int* __restrict__ row_state, int reduction,
                                                  float* __restrict__ loss, float* __restrict__ inv_count,
                                                  int* __restrict__ correct, int* __restrict__ status) {
  __shared__ float rl[256];
  __shared__ int rc[256], rk[256], rb[256];
  float l = 0.f;
  int cnt = 0, ok = 0, bad = 0;
  for (int i = threadIdx.x; i < N; i += 256) {
    const int st = row_state[i];
    if (st & 3) { l += row_loss[i]; cnt += 1; }
    ok += (st >> 2) & 1;
    bad |= (st & 3) == 2;
  }
  rl[threadIdx.x] = l; rc[threadIdx.x] = cnt; rk[threadIdx.x] = ok; rb[threadIdx.x] = bad;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      rl[threadIdx.x] += rl[threadIdx.x + s];
      rc[threadIdx.x] += rc[threadIdx.x + s];
      rk[threadIdx.x] += rk[threadIdx.x + s];
      rb[threadIdx.x] |= rb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float inv = reduction == 1 ? (rc[0] > 0 ? 1.f / (float)rc[0] : NAN) : 1.f;   // torch: mean of nothing = nan
    if (loss) *loss = reduction == 1 ? rl[0] * inv : rl[0];
    if (inv_count) *inv_count = inv;
    if (correct) *correct = rk[0];
    if (status) *status = rb[0];
  }
}

// dz[r][c] (strides d_row, d_col) = beta·dz + scale·g·dloss_r/dz_rc with g = g_up[r] for reduction 'none'
// (per-row upstream gradients) and g = (*g_up or 1)·(1/count or 1) for 'mean' / 'sum'.
__global__ __launch_bounds__(256) void xent_grad(int N, int C, const float* __restrict__ L, long s_row, long s_col,
                                                 const long* __restrict__ labels, long ignore_index, float eps,
                                                 float gamma, float alpha, const float* __restrict__ inv_count,
                                                 const float* __restrict__ g_up, int per_row, float scale, float beta,
                                                 float* __restrict__ dZ, long d_row, long d_col) {
  const int row = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* z = L + (long)row * s_row;
  float* dz = dZ + (long)row * d_row;
  const long y = labels ? labels[row] : (long)row;
  const bool skip = y == ignore_index || y < 0 || y >= C;
  float m = -INFINITY;
  for (int j = lane; j < C; j += 64) m = fmaxf(m, z[(long)j * s_col]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  float s = 0.f, sz = 0.f;
  for (int j = lane; j < C; j += 64) {
    const float v = z[(long)j * s_col];
    s += __expf(v - m);
    sz += v;
  }
  s = wave_sum(s);
  sz = wave_sum(sz);
  const float lse = m + __logf(s);
  float w_q = alpha, w_h = 0.f;                 // dz = w_q·(p - q) + w_h·(p - onehot)
  if (!skip && gamma != 0.f) {
    const float zy = z[y * s_col];
    const float ce = (1.f - eps) * (lse - zy) + eps * (lse - sz / (float)C);
    const float pt = __expf(-ce), om = fmaxf(1.f - pt, 0.f);
    w_q = alpha * __powf(om, gamma);
    w_h = om > 0.f ? alpha * gamma * __powf(om, gamma - 1.f) * pt * ce : 0.f;
  }
  const float g = skip ? 0.f : scale * (per_row ? g_up[row] : (g_up ? *g_up : 1.f) * *inv_count);
  for (int j = lane; j < C; j += 64) {
    const float p = __expf(z[(long)j * s_col] - lse);
    const float oh = (j == y) ? 1.f : 0.f;
    const float q = (1.f - eps) * oh + eps / (float)C;
    float v = g * (w_q * (p - q) + w_h * (p - oh));
    float* o = dz + (long)j * d_col;
    if (beta != 0.f) v += beta * *o;
    *o = v;
  }
}

}  // namespace

extern "C" long cmhar_cross_entropy_ws(int N) { return 2L * N + 8; }

extern "C" int cmhar_cross_entropy(int N, int C, const float* logits, long s_row, long s_col, const long* labels,
                                   long ignore_index, float label_smoothing, float gamma, float alpha, int reduction,
                                   float* loss, float* row_loss, long* pred, int* correct, int* status,
                                   float* dlogits, long d_row, long d_col, float grad_scale, float grad_beta,
                                   const float* g_up, float* ws, hipStream_t st) {
  if (N <= 0) return 0;
  if (C <= 0 || reduction < 0 || reduction > 2 || (gamma != 0.f && label_smoothing != 0.f)) return -1;
  if (dlogits && reduction == 0 && !g_up) return -2;
  float* rl = row_loss ? row_loss : ws;
  int* rs = (int*)(ws + N);
  float* inv = ws + 2L * N;
  const int blocks = cdiv((long)N * 64, 256);
  xent_rows<<<blocks, 256, 0, st>>>(N, C, logits, s_row, s_col, labels, ignore_index, label_smoothing, gamma, alpha,
                                    rl, rs, pred);
  xent_final<<<1, 256, 0, st>>>(N, rl, rs, reduction, loss, inv, correct, status);
  if (dlogits)
    xent_grad<<<blocks, 256, 0, st>>>(N, C, logits, s_row, s_col, labels, ignore_index, label_smoothing, gamma, alpha,
                                      inv, g_up, reduction == 0, grad_scale, grad_beta, dlogits, d_row, d_col);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

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
