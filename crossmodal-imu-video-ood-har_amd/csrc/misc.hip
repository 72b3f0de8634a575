// Data-movement kernels around the hot path: tubelet patch extraction (VideoMAE Conv3d as GEMM), the IMU
// PatchTST embedding, strided copies with dtype conversion, and the multi-tensor optimizer step
// (clip_grad_norm_ + AdamW, trainer.py:138-141) with fused bf16 shadow-weight refresh.
#include "common.h"
#include <algorithm>

namespace {

// video (B, T, C, H, W) fp32 → patches [B*L][C*tub*P*P] (row order (t', h', w'), column order (c, dt, dy, dx) —
// the flatten order of Conv3d weight [hidden, C, tub, P, P], modeling_videomae.py:159-168).
template <typename TO>
__global__ void tubelet_im2col_kernel(int B, int T, int C, int H, int W, int tub, int P, const float* __restrict__ v,
                                      TO* __restrict__ out) {
  const int Tp = T / tub, Hp = H / P, Wp = W / P;
  const long L = (long)Tp * Hp * Wp;
  const int K = C * tub * P * P;
  const int groups = P / 8;                  // 8 consecutive dx per thread
  const long total = (long)B * L * C * tub * P * groups;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  long r = idx;
  const int gx = r % groups; r /= groups;
  const int dy = r % P; r /= P;
  const int dt = r % tub; r /= tub;
  const int c = r % C; r /= C;
  const long tok = r % L;
  const int b = r / L;
  const int wp = tok % Wp, hp = (tok / Wp) % Hp, tp = tok / ((long)Wp * Hp);
  const float* src = v + ((((long)b * T + tp * tub + dt) * C + c) * H + hp * P + dy) * W + wp * P + gx * 8;
  TO* dst = out + ((long)b * L + tok) * K + ((c * tub + dt) * P + dy) * P + gx * 8;
  const floatx4 x0 = *(const floatx4*)src, x1 = *(const floatx4*)(src + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { dst[j] = from_f<TO>(x0[j]); dst[4 + j] = from_f<TO>(x1[j]); }
}

struct PtrTable8 { const float* p[8]; };
struct MutPtrTable8 { float* p[8]; };

// IMU PatchTST embedding + CLS + positional table, truncated to T tokens (models.py:40-49, 115-123).
// token 0 = cls + pos[0]; token 1+t (t < T-1) = channel c = t / N, patch n = t % N.
__global__ void imu_embed_fwd_kernel(int B, int C, int L, int N, int P, int S, int D, int T,
                                     const float* __restrict__ x, PtrTable8 w, PtrTable8 bias,
                                     const float* __restrict__ cls, const float* __restrict__ pos,
                                     float* __restrict__ out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * T * D) return;
  const int d = idx % D;
  const int tok = (idx / D) % T;
  const int b = idx / ((long)D * T);
  float v;
  if (tok == 0) v = cls[d];
  else {
    const int t = tok - 1, c = t / N, n = t % N;
    const float* xs = x + ((long)b * C + c) * L + (long)n * S;
    const float* wr = w.p[c] + (long)d * P;
    v = bias.p[c][d];
    for (int p = 0; p < P; ++p) v = fmaf(xs[p], wr[p], v);
  }
  out[idx] = v + pos[(long)tok * D + d];
}

// Gradients: dcls, dpos[0:T] (rest of the table untouched → zero), dW_c, db_c (channels without live tokens → 0).
// blockIdx.y = 0: dpos[tok, d] = Σ_b dout[b, tok, d] (tok < T; rows past the used length get 0) and dcls = dpos[0];
// blockIdx.y = 1 + c: one thread per (d, p) of channel c's Linear(P → D): dW[d, p] = Σ_{n, b} dout[b, tok, d]·x[b, c,
// nS + p] over the channel's tokens that survive the pos-table truncation (models.py:122-123: channels 1.. get
// exact zeros), and the p == 0 threads also form the bias gradient.
__global__ __launch_bounds__(256) void imu_embed_bwd_kernel(int B, int C, int L, int N, int P, int S, int D, int T,
                                                            int Tpos, const float* __restrict__ x,
                                                            const float* __restrict__ dout, float* __restrict__ dcls,
                                                            float* __restrict__ dpos, MutPtrTable8 dw,
                                                            MutPtrTable8 db) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y == 0) {
    if (idx >= Tpos * D) return;
    const int tok = idx / D, d = idx % D;
    float s = 0.f;
    if (tok < T)
      for (int b = 0; b < B; ++b) s += dout[((long)b * T + tok) * D + d];
    dpos[(long)tok * D + d] = s;
    if (tok == 0) dcls[d] = s;
    return;
  }
  if (idx >= D * P) return;
  const int c = blockIdx.y - 1, d = idx / P, p = idx % P;
  float gw = 0.f, gb = 0.f;
  for (int n = 0; n < N; ++n) {
    const int tok = 1 + c * N + n;
    if (tok >= T) break;
#pragma unroll 4
    for (int b = 0; b < B; ++b) {
      const float g = dout[((long)b * T + tok) * D + d];
      gb += g;
      gw = fmaf(g, x[((long)b * C + c) * L + (long)n * S + p], gw);
    }
  }
  dw.p[c][(long)d * P + p] = gw;
  if (p == 0) db.p[c][d] = gb;
}

// dst = alpha * src * dropmask(seed, p, r, c) + beta * dst   (dropout forward/backward, casts, adds, gathers)
template <typename TI, typename TO>
__global__ void copy2d_kernel(int rows, int cols, const TI* __restrict__ src, long lds, TO* __restrict__ dst,
                              long ldd, float alpha, float beta, float pdrop, unsigned long long seed) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)rows * cols) return;
  const int r = idx / cols, c = idx % cols;
  float v = alpha * to_f<TI>(src[(long)r * lds + c]);
  if (pdrop > 0.f) v *= drop_mask(seed, pdrop, r, c);
  TO* d = dst + (long)r * ldd + c;
  if (beta != 0.f) v += beta * to_f<TO>(*d);
  *d = from_f<TO>(v);
}

// ---------------------------------------------------------------------------------------------------------------
// multi-tensor optimizer kernels.  Tensor table entries + a chunk list (built on the host once per step).
// ---------------------------------------------------------------------------------------------------------------
struct MTTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16* pbf;      // optional bf16 compute shadow (nullable)
  float* pcopy;   // optional fp32 compute copy (nullable), e.g. a slice of a packed QKV bias
  long n;
  float wd;       // per-tensor weight decay
  float lr_scale; // per-group lr multiplier
};
struct MTChunk {
  int t;
  int pad;
  long start;
  long len;
};

__global__ __launch_bounds__(256) void mt_sqnorm_kernel(const MTTensor* __restrict__ tens,
                                                        const MTChunk* __restrict__ chunks, float* __restrict__ part) {
  const MTChunk ch = chunks[blockIdx.x];
  const float* g = tens[ch.t].g;
  float s = 0.f;
  if (g) {
    for (long i = ch.start + threadIdx.x * 4; i < ch.start + ch.len; i += 1024) {
      if (i + 3 < ch.start + ch.len) {
        const floatx4 x = *(const floatx4*)(g + i);
        s += x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
      } else {
        for (long j = i; j < ch.start + ch.len; ++j) s += g[j] * g[j];
      }
    }
  }
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// total norm → out[0] = norm, out[1] = clip coefficient clamped to 1 (torch clip_grad_norm_ semantics).
__global__ void mt_norm_final_kernel(int nparts, const float* __restrict__ part, float* __restrict__ out,
                                     float max_norm) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float n = (float)sqrt(red[0]);
    out[0] = n;
    out[1] = fminf(max_norm / (n + 1e-6f), 1.f);
  }
}

__global__ __launch_bounds__(256) void mt_scale_kernel(const MTTensor* __restrict__ tens,
                                                       const MTChunk* __restrict__ chunks,
                                                       const float* __restrict__ coef) {
  const MTChunk ch = chunks[blockIdx.x];
  float* g = (float*)tens[ch.t].g;
  if (!g) return;
  const float c = coef[1];
  for (long i = ch.start + threadIdx.x; i < ch.start + ch.len; i += 256) g[i] *= c;
}

// torch.optim.AdamW math order (lerp for exp_avg, mul+addcmul for exp_avg_sq, denom = sqrt(v)/sqrt(bc2) + eps,
// p *= 1 - lr*wd, p += -step_size * m/denom).  All step scalars are computed by the host in double precision, as
// torch does in Python floats.  Optional grad scale from device memory (clip coefficient, out[1]); with write_g the
// scaled gradient is stored back (the clipped .grad of clip_grad_norm_, produced in the same pass); bf16 shadow.
// Four elements per thread-iteration when every stream of the tensor is 16-B aligned (8-B for the bf16 shadow) —
// the same per-element arithmetic as the scalar loop.
// g·scale rounded to fp32 as its own instruction: no FMA contraction into the moment updates (the folded clip must
// see exactly the value a separate scale pass would have stored).  (__fmul_rn alone still contracted.)
__device__ __forceinline__ float mul_nocontract(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}

__device__ __forceinline__ void adamw_elem(float g, float& p, float& m, float& v, float decay, float omb1,
                                           float beta2, float omb2, float eps, float ss, float bc2_sqrt) {
  p = p * decay;
  m = m + omb1 * (g - m);
  v = beta2 * v + omb2 * (g * g);
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + (-ss) * (m / denom);
}

__global__ __launch_bounds__(256) void mt_adamw_kernel(const MTTensor* __restrict__ tens,
                                                       const MTChunk* __restrict__ chunks, float lr, float omb1,
                                                       float beta2, float omb2, float eps, float step_size,
                                                       float bc2_sqrt, const float* __restrict__ gscale, int write_g) {
  const MTChunk ch = chunks[blockIdx.x];
  const MTTensor T = tens[ch.t];
  if (!T.g) return;
  const float gs = gscale ? gscale[1] : 1.f;
  const bool wg = write_g && gscale;
  const float ss = step_size * T.lr_scale;
  const float decay = 1.f - lr * T.lr_scale * T.wd;
  float* G = const_cast<float*>(T.g);
  const unsigned long al = (unsigned long)T.p | (unsigned long)T.g | (unsigned long)T.m | (unsigned long)T.v |
                           (unsigned long)T.pcopy;
  const bool vec = (al & 15) == 0 && ((unsigned long)T.pbf & 7) == 0 && (ch.start & 3) == 0;
  long i0 = ch.start;
  const long end = ch.start + ch.len;
  if (vec) {
    const long nv = (ch.len >> 2) << 2;
    // two float4 groups per thread per iteration, all eight loads issued before the first store (more bytes in
    // flight per thread: the pass is HBM-latency bound at one group)
    auto step4 = [&](long i, floatx4 g4, floatx4 p4, floatx4 m4, floatx4 v4) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g4[j] = mul_nocontract(g4[j], gs);     // rounded product (no FMA contraction): the value a scale pass would store
        float pj = p4[j], mj = m4[j], vj = v4[j];
        adamw_elem(g4[j], pj, mj, vj, decay, omb1, beta2, omb2, eps, ss, bc2_sqrt);
        p4[j] = pj; m4[j] = mj; v4[j] = vj;
      }
      *(floatx4*)(T.p + i) = p4;
      *(floatx4*)(T.m + i) = m4;
      *(floatx4*)(T.v + i) = v4;
      if (wg) *(floatx4*)(G + i) = g4;
      if (T.pbf) {
        bf16 __attribute__((ext_vector_type(4))) b4;
#pragma unroll
        for (int j = 0; j < 4; ++j) b4[j] = (bf16)p4[j];
        *(decltype(b4)*)(T.pbf + i) = b4;
      }
      if (T.pcopy) *(floatx4*)(T.pcopy + i) = p4;
    };
    long i = ch.start + threadIdx.x * 4;
    for (; i + 1024 < ch.start + nv; i += 2048) {
      const floatx4 ga = *(const floatx4*)(T.g + i), pa = *(const floatx4*)(T.p + i);
      const floatx4 ma = *(const floatx4*)(T.m + i), va = *(const floatx4*)(T.v + i);
      const floatx4 gb = *(const floatx4*)(T.g + i + 1024), pb = *(const floatx4*)(T.p + i + 1024);
      const floatx4 mb = *(const floatx4*)(T.m + i + 1024), vb = *(const floatx4*)(T.v + i + 1024);
      step4(i, ga, pa, ma, va);
      step4(i + 1024, gb, pb, mb, vb);
    }
    if (i < ch.start + nv)
      step4(i, *(const floatx4*)(T.g + i), *(const floatx4*)(T.p + i), *(const floatx4*)(T.m + i),
            *(const floatx4*)(T.v + i));
    i0 = ch.start + nv;
  }
  for (long i = i0 + threadIdx.x; i < end; i += 256) {
    const float g = mul_nocontract(T.g[i], gs);
    float p = T.p[i], m = T.m[i], v = T.v[i];
    adamw_elem(g, p, m, v, decay, omb1, beta2, omb2, eps, ss, bc2_sqrt);
    T.p[i] = p;
    T.m[i] = m;
    T.v[i] = v;
    if (wg) G[i] = g;
    if (T.pbf) T.pbf[i] = (bf16)p;
    if (T.pcopy) T.pcopy[i] = p;
  }
}

__global__ __launch_bounds__(256) void mt_cast_kernel(const MTTensor* __restrict__ tens,
                                                      const MTChunk* __restrict__ chunks) {
  const MTChunk ch = chunks[blockIdx.x];
  const MTTensor T = tens[ch.t];
  for (long i = ch.start + threadIdx.x; i < ch.start + ch.len; i += 256) {
    const float x = T.p[i];
    if (T.pbf) T.pbf[i] = (bf16)x;
    if (T.pcopy) T.pcopy[i] = x;
  }
}

// Transposed bf16 weight shadows (the input-gradient GEMMs read Wᵀ [K, N] K-contiguous in the forward layout instead
// of W [N, K] through transposed LDS reads).  One launch over every matrix: a workgroup transposes one 64×64 tile,
// read as 16-B row pieces (coalesced), staged in LDS with a padded row pitch, written as 16-B row pieces of the
// destination.  rows, cols multiples of 8; a descriptor's tiles start at `tile0` (prefix sums, ascending).
struct MTTranspose {
  const bf16* src;
  bf16* dst;
  int rows, cols;     // source shape [rows, cols], row-major; destination [cols, rows]
  int tile0, pad;
};

__global__ __launch_bounds__(256) void mt_transpose_kernel(const MTTranspose* __restrict__ descs, int ndesc) {
  __shared__ unsigned short tile[64][64 + 8];
  int d = 0;
  while (d + 1 < ndesc && descs[d + 1].tile0 <= (int)blockIdx.x) ++d;
  const MTTranspose D = descs[d];
  const int t = blockIdx.x - D.tile0;
  const int tiles_c = (D.cols + 63) / 64;
  const int r0 = (t / tiles_c) * 64, c0 = (t % tiles_c) * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {          // 64 rows × 8 pieces of 16 B
    const int piece = tid + 256 * i, r = piece >> 3, cp = (piece & 7) * 8;
    uint4_t v = {0u, 0u, 0u, 0u};
    if (r0 + r < D.rows && c0 + cp < D.cols) v = *(const uint4_t*)(D.src + (long)(r0 + r) * D.cols + c0 + cp);
    *(uint4_t*)&tile[r][cp] = v;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {          // destination rows = source columns
    const int piece = tid + 256 * i, c = piece >> 3, rp = (piece & 7) * 8;
    if (c0 + c >= D.cols || r0 + rp >= D.rows) continue;
    unsigned short e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[rp + j][c];
    uint4_t v = {e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16), e[4] | ((unsigned)e[5] << 16),
                 e[6] | ((unsigned)e[7] << 16)};
    *(uint4_t*)(D.dst + (long)(c0 + c) * D.rows + r0 + rp) = v;
  }
}

}  // namespace

extern "C" int cmhar_mt_transpose_bf16(const void* descs, int ndesc, int ntiles, hipStream_t st) {
  if (ndesc <= 0 || ntiles <= 0) return 0;
  mt_transpose_kernel<<<ntiles, 256, 0, st>>>((const MTTranspose*)descs, ndesc);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_tubelet_im2col(int out_dtype, int B, int T, int C, int H, int W, int tub, int P,
                                    const float* video, void* out, hipStream_t st) {
  if (P % 8 != 0 || T % tub || H % P || W % P) return -1;
  const long total = (long)B * (T / tub) * (H / P) * (W / P) * C * tub * P * (P / 8);
  if (total == 0) return 0;
  if (out_dtype == CMHAR_BF16)
    tubelet_im2col_kernel<bf16><<<cdiv(total, 256), 256, 0, st>>>(B, T, C, H, W, tub, P, video, (bf16*)out);
  else if (out_dtype == CMHAR_F16)
    tubelet_im2col_kernel<f16><<<cdiv(total, 256), 256, 0, st>>>(B, T, C, H, W, tub, P, video, (f16*)out);
  else
    tubelet_im2col_kernel<float><<<cdiv(total, 256), 256, 0, st>>>(B, T, C, H, W, tub, P, video, (float*)out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_imu_embed_fwd(int B, int C, int L, int N, int P, int S, int D, int T, const float* x,
                                   const float* const* w, const float* const* bias, const float* cls, const float* pos,
                                   float* out, hipStream_t st) {
  if (C > 8 || P > 32) return -1;
  PtrTable8 tw{}, tb{};
  for (int c = 0; c < C; ++c) { tw.p[c] = w[c]; tb.p[c] = bias[c]; }
  const long total = (long)B * T * D;
  imu_embed_fwd_kernel<<<cdiv(total, 256), 256, 0, st>>>(B, C, L, N, P, S, D, T, x, tw, tb, cls, pos, out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_imu_embed_bwd(int B, int C, int L, int N, int P, int S, int D, int T, int Tpos, const float* x,
                                   const float* dout, float* dcls, float* dpos, float* const* dw, float* const* db,
                                   hipStream_t st) {
  if (C > 8) return -1;
  MutPtrTable8 tw{}, tb{};
  for (int c = 0; c < C; ++c) { tw.p[c] = dw[c]; tb.p[c] = db[c]; }
  const int nblk = cdiv(std::max(D * P, Tpos * D), 256);
  imu_embed_bwd_kernel<<<dim3(nblk, C + 1), 256, 0, st>>>(B, C, L, N, P, S, D, T, Tpos, x, dout, dcls, dpos, tw, tb);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_copy2d(int in_dtype, int out_dtype, int rows, int cols, const void* src, long lds, void* dst,
                            long ldd, float alpha, float beta, float pdrop, unsigned long long seed,
                            hipStream_t st) {
  const long total = (long)rows * cols;
  if (total == 0) return 0;
  const int g = cdiv(total, 256);
#define C2(TI, TO)                                                                                          \
  copy2d_kernel<TI, TO><<<g, 256, 0, st>>>(rows, cols, (const TI*)src, lds, (TO*)dst, ldd, alpha, beta, pdrop, \
                                           seed)
  if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_F32) C2(float, float);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_BF16) C2(float, bf16);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_F32) C2(bf16, float);
  else if (in_dtype == CMHAR_F16 && out_dtype == CMHAR_F32) C2(f16, float);
  else if (in_dtype == CMHAR_F32 && out_dtype == CMHAR_F16) C2(float, f16);
  else if (in_dtype == CMHAR_F16 && out_dtype == CMHAR_F16) C2(f16, f16);
  else if (in_dtype == CMHAR_BF16 && out_dtype == CMHAR_BF16) C2(bf16, bf16);
  else return -1;
#undef C2
  CMHAR_CHECK_LAUNCH();
  return 0;
}

// Multi-tensor entry points: `tens` / `chunks` are DEVICE arrays (MTTensor / MTChunk layouts above).
extern "C" int cmhar_mt_grad_norm(const void* tens, const void* chunks, int nchunks, float* part, float* out,
                                  float max_norm, int apply_clip, hipStream_t st) {
  if (nchunks <= 0) return 0;
  mt_sqnorm_kernel<<<nchunks, 256, 0, st>>>((const MTTensor*)tens, (const MTChunk*)chunks, part);
  mt_norm_final_kernel<<<1, 256, 0, st>>>(nchunks, part, out, max_norm);
  if (apply_clip) mt_scale_kernel<<<nchunks, 256, 0, st>>>((const MTTensor*)tens, (const MTChunk*)chunks, out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_mt_adamw(const void* tens, const void* chunks, int nchunks, float lr, float omb1, float beta2,
                              float omb2, float eps, float step_size, float bc2_sqrt, const float* gscale,
                              hipStream_t st) {
  return cmhar_mt_adamw_clip(tens, chunks, nchunks, lr, omb1, beta2, omb2, eps, step_size, bc2_sqrt, gscale, 0, st);
}

extern "C" int cmhar_mt_adamw_clip(const void* tens, const void* chunks, int nchunks, float lr, float omb1,
                                   float beta2, float omb2, float eps, float step_size, float bc2_sqrt,
                                   const float* gscale, int write_grad, hipStream_t st) {
  if (nchunks <= 0) return 0;
  mt_adamw_kernel<<<nchunks, 256, 0, st>>>((const MTTensor*)tens, (const MTChunk*)chunks, lr, omb1, beta2, omb2, eps,
                                           step_size, bc2_sqrt, gscale, write_grad);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_mt_cast_bf16(const void* tens, const void* chunks, int nchunks, hipStream_t st) {
  if (nchunks <= 0) return 0;
  mt_cast_kernel<<<nchunks, 256, 0, st>>>((const MTTensor*)tens, (const MTChunk*)chunks);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int cmhar_version(void) { return 1; }
