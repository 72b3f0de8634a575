// Ingestion kernels: the steps on either side of the hot path's inputs.
//
// 1. Video clip ingestion (replaces: CrossModalDataset.load_video_clip, src/data/datasets.py:155-235, and its
//    transform, :49-58 — ToPILImage → Resize(video_resize) → ToTensor → Normalize(ImageNet)).  Input: decoded RGB
//    uint8 frames [nf][H0][W0][3] resident in HBM (decoding itself is out of scope: cv2 is absent here) and, per
//    clip, the T source-frame indices the reference picks (np.linspace over the 5 s window, computed by the host).
//    Output: the normalised clip batch, fp32 (B,T,3,H,W) or (B,3,T,H,W) — exactly what the model consumes.
//    The resize is Pillow's BILINEAR resample (what torchvision's Resize does to a PIL image), restated bit-exactly:
//    triangle filter widened by the downscale factor (antialias), coefficients computed in double and quantised to
//    22-bit fixed point, a horizontal pass rounding to uint8, then a vertical pass rounding to uint8 (Pillow
//    src/libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc, ImagingResample{Horizontal,Vertical}_8bpc).
//    Then v/255 and (v - mean)/std in fp32, as ToTensor / Normalize do.  All integer until the last step: HBM-bound.
//
// 2. IMU preprocessing (replaces: MMEAPreprocessor.load_imu_data unit conversion, preprocess_imu and
//    create_imu_windows, src/data/preprocessing.py:176-183, 204-243).  Input: a ragged batch of recordings
//    (concatenated [total][C] fp32 raw samples + offsets).  Per recording and channel: optional raw/R unit scale,
//    median filter of width k (scipy.signal.medfilt: zero padding at both ends), z-score with the population
//    std + 1e-8 (divisions, not reciprocal products, so fp32 rounding matches numpy's), then windows of `win`
//    samples every `stride` (short recordings zero-padded to one window), written channel-major (C, win) — the
//    layout load_imu_window hands to the model (datasets.py:108-140).
#include "common.h"

namespace {

constexpr int PREC = 22;                       // Pillow PRECISION_BITS = 32 - 8 - 2

// Pillow precompute_coeffs + normalize_coeffs_8bpc for one output coordinate.  Plain double arithmetic with FMA
// contraction off, so the quantised coefficients are those of Pillow's C build.
#pragma clang fp contract(off)
__global__ void resize_coeffs_kernel(int in_size, int out_size, int ksize, int* __restrict__ bounds,
                                     int* __restrict__ kk) {
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= out_size) return;
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[64];
  double ww = 0.0;
  for (int x = 0; x < xmax && x < 64; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    const double f = t < 1.0 ? 1.0 - t : 0.0;
    w[x] = f;
    ww += f;
  }
  for (int x = 0; x < ksize; ++x) {
    double k = 0.0;
    if (x < xmax) k = ww != 0.0 ? w[x] / ww : w[x];
    kk[(long)xx * ksize + x] = k < 0 ? (int)(-0.5 + k * (1 << PREC)) : (int)(0.5 + k * (1 << PREC));
  }
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = xmax;
}
#pragma clang fp contract(on)

__device__ __forceinline__ unsigned char clip8(int v) {
  if (v >= (1 << PREC << 8)) return 255;
  if (v <= 0) return 0;
  return (unsigned char)(v >> PREC);
}

// Horizontal pass: tmp[f][y - y0][xx] = packed RGBX (uint32) for source rows y0 <= y < y0 + rows of frame idx[f].
// A workgroup owns R consecutive source rows of one frame: it stages them into LDS widened to one 32-bit word per
// pixel (three 16-B loads = 16 pixels per thread when rows are 16-B aligned, byte loads otherwise), then each
// thread computes one output column for all R rows from ds_read_b32 taps.  One HBM read of each source byte.
__global__ __launch_bounds__(256) void resize_h_kernel(const unsigned char* __restrict__ frames, long frame_stride,
                                                       int W0, const int* __restrict__ idx, int y0, int rows, int R,
                                                       int W, int ksize, const int* __restrict__ bounds,
                                                       const int* __restrict__ kk, unsigned* __restrict__ tmp,
                                                       int aligned) {
  extern __shared__ unsigned px[];                        // [R][W0] RGBX
  const int f = blockIdx.y;
  const int r0 = blockIdx.x * R;
  const int nr = min(R, rows - r0);
  const unsigned char* src = frames + (long)idx[f] * frame_stride + (long)(y0 + r0) * W0 * 3;
  if (aligned) {                                          // 16 pixels = 48 B = 3 x 16-B loads per thread
    const int g16 = W0 / 16, ng = nr * g16;
    for (int g = threadIdx.x; g < ng; g += blockDim.x) {
      const int r = g / g16, q = g % g16;
      const uint4_t* p = (const uint4_t*)(src + (long)r * W0 * 3 + q * 48);
      const uint4_t u0 = p[0], u1 = p[1], u2 = p[2];
      const unsigned w[12] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3], u2[0], u2[1], u2[2], u2[3]};
      unsigned* o = px + r * W0 + q * 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {                       // 3 words = 4 pixels: r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
        const unsigned a = w[3 * j], b = w[3 * j + 1], c = w[3 * j + 2];
        o[4 * j + 0] = a & 0xffffffu;
        o[4 * j + 1] = (a >> 24) | ((b & 0xffffu) << 8);
        o[4 * j + 2] = (b >> 16) | ((c & 0xffu) << 16);
        o[4 * j + 3] = c >> 8;
      }
    }
  } else {
    const int n = nr * W0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int r = i / W0, x = i % W0;
      const unsigned char* p = src + (long)r * W0 * 3 + x * 3;
      px[i] = p[0] | (p[1] << 8) | (p[2] << 16);
    }
  }
  __syncthreads();
  // one output column per thread for all of the workgroup's rows: its taps / coefficients are loaded once
  for (int xx = threadIdx.x; xx < W; xx += blockDim.x) {
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int* k = kk + (long)xx * ksize;
    for (int r = 0; r < nr; ++r) {
      const unsigned* row = px + r * W0 + xmin;
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;        // Pillow's INT32 sums: < 2^31 (bilinear weights >= 0)
      for (int x = 0; x < xmax; ++x) {
        const unsigned v = row[x];
        const unsigned kx = (unsigned)k[x];               // <= 2^22: 24-bit multiplies are exact
        s0 += __umul24(v & 0xff, kx);
        s1 += __umul24((v >> 8) & 0xff, kx);
        s2 += __umul24((v >> 16) & 0xff, kx);
      }
      tmp[((long)f * rows + r0 + r) * W + xx] = clip8(s0) | (clip8(s1) << 8) | (clip8(s2) << 16);
    }
  }
}

// Vertical pass + ToTensor + Normalize: one thread per output pixel (yy, xx) of frame f, all three channels.
__global__ __launch_bounds__(256) void resize_v_norm_kernel(const unsigned* __restrict__ tmp, int rows, int y0,
                                                            int H, int W, int ksize, const int* __restrict__ bounds,
                                                            const int* __restrict__ kk, float m0, float m1, float m2,
                                                            float s0, float s1, float s2, int T, int channel_first,
                                                            float* __restrict__ out) {
  const int f = blockIdx.y;
  const long n = (long)H * W;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int yy = (int)(i / W), xx = (int)(i % W);
  const int ymin = bounds[2 * yy] - y0, ymax = bounds[2 * yy + 1];
  const int* k = kk + (long)yy * ksize;
  const unsigned* src = tmp + (long)f * rows * W + xx;
  int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
  for (int y = 0; y < ymax; ++y) {
    const unsigned v = src[(long)(ymin + y) * W];        // coalesced across xx
    const unsigned ky = (unsigned)k[y];
    a0 += __umul24(v & 0xff, ky);
    a1 += __umul24((v >> 8) & 0xff, ky);
    a2 += __umul24((v >> 16) & 0xff, ky);
  }
  const float v0 = (float)clip8(a0) / 255.f, v1 = (float)clip8(a1) / 255.f, v2 = (float)clip8(a2) / 255.f;
  const int b = f / T, t = f % T;
  const long plane = (long)H * W;
  // (B,T,3,H,W): channel stride plane, frame stride 3 plane;  (B,3,T,H,W): channel stride T plane, frame stride plane
  const long cs = channel_first ? (long)T * plane : plane;
  float* o = out + (long)b * T * 3 * plane + (channel_first ? (long)t * plane : (long)t * 3 * plane) + i;
  o[0] = (v0 - m0) / s0;
  o[cs] = (v1 - m1) / s1;
  o[2 * cs] = (v2 - m2) / s2;
}

// ---------------------------------------------------------------------------------------------------------------
// IMU preprocessing.  Stage 1: one workgroup per (recording, channel): scaled + median-filtered series into tmp,
// then mean / population std of the filtered series (two passes over tmp: the same two-pass formula numpy uses).
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int j = 0; j < (int)(blockDim.x >> 6); ++j) s += red[j];
  return s;
}

__global__ __launch_bounds__(256) void imu_filter_stats_kernel(const float* __restrict__ raw,
                                                               const long* __restrict__ offsets, int C, int k,
                                                               const float* __restrict__ div_r, int normalize,
                                                               float* __restrict__ filt, float* __restrict__ mean,
                                                               float* __restrict__ sd) {
  __shared__ float red[4];
  const int rec = blockIdx.x, c = blockIdx.y;
  const long o0 = offsets[rec], n = offsets[rec + 1] - o0;
  const float r = div_r ? div_r[c] : 1.f;
  const int h = k / 2;
  float acc = 0.f;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    float v;
    if (k > 1) {
      float win[65];
      for (int j = -h; j <= h; ++j) {                     // zero padding outside the recording (medfilt)
        const long q = i + j;
        win[j + h] = (q >= 0 && q < n) ? raw[(o0 + q) * C + c] / r : 0.f;
      }
      for (int a = 1; a < k; ++a) {                       // insertion sort of k <= 65 values: exact median
        const float x = win[a];
        int b = a - 1;
        while (b >= 0 && win[b] > x) { win[b + 1] = win[b]; --b; }
        win[b + 1] = x;
      }
      v = win[h];
    } else {
      v = raw[(o0 + i) * C + c] / r;
    }
    filt[(o0 + i) * C + c] = v;
    acc += v;
  }
  const float mu = n > 0 ? block_sum(acc, red) / (float)n : 0.f;
  float acc2 = 0.f;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = filt[(o0 + i) * C + c] - mu;
    acc2 += d * d;
  }
  const float var = n > 0 ? block_sum(acc2, red) / (float)n : 0.f;
  if (threadIdx.x == 0) {
    mean[rec * C + c] = normalize ? mu : 0.f;
    sd[rec * C + c] = normalize ? sqrtf(var) + 1e-8f : 1.f;
  }
}

// Stage 2: windows.  One thread per output element (window, channel, t): out[w][c][t] = z(filt[start + t]) or 0
// past the end of a short (padded) recording.
__global__ __launch_bounds__(256) void imu_window_kernel(const float* __restrict__ filt,
                                                         const long* __restrict__ offsets,
                                                         const int* __restrict__ win_rec,
                                                         const long* __restrict__ win_start, int C, int win,
                                                         const float* __restrict__ mean, const float* __restrict__ sd,
                                                         long nwin, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nwin * C * win) return;
  const int t = (int)(i % win);
  const int c = (int)((i / win) % C);
  const long w = i / ((long)win * C);
  const int rec = win_rec[w];
  const long n = offsets[rec + 1] - offsets[rec];
  const long q = win_start[w] + t;
  // preprocess_imu z-scores the filtered series, then create_imu_windows pads the NORMALISED series with zeros
  out[i] = q < n ? (filt[(offsets[rec] + q) * C + c] - mean[rec * C + c]) / sd[rec * C + c] : 0.f;
}

}  // namespace

extern "C" int cmhar_resize_ksize(int in_size, int out_size) {
  const double scale = (double)in_size / (double)out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)ceil(support) * 2 + 1;
}

extern "C" long cmhar_video_ingest_ws(int nframes, int H0, int W0, int H, int W) {
  const int kh = cmhar_resize_ksize(W0, W), kv = cmhar_resize_ksize(H0, H);
  const long ints = 2L * W + (long)W * kh + 2L * H + (long)H * kv;
  const long tmp_bytes = (long)nframes * H0 * W * 4;      // RGBX words; upper bound of the horizontal pass' rows
  return ints * 4 + tmp_bytes + 64;
}

extern "C" int cmhar_video_ingest(int B, int T, const unsigned char* frames, long frame_stride, int H0, int W0,
                                  const int* frame_idx, int H, int W, const float* mean3, const float* std3,
                                  int channel_first, float* out, void* ws, long ws_bytes, hipStream_t st) {
  if (B <= 0 || T <= 0) return 0;
  if (H0 <= 0 || W0 <= 0 || H <= 0 || W <= 0 || frame_stride < (long)H0 * W0 * 3) return -1;
  const int kh = cmhar_resize_ksize(W0, W), kv = cmhar_resize_ksize(H0, H);
  if (kh > 64 || kv > 64) return -2;                      // downscale factor > 31: not supported
  if (W0 > 16384) return -4;                              // one source row must fit the LDS stage
  if (ws_bytes < cmhar_video_ingest_ws(B * T, H0, W0, H, W)) return -3;
  int* bh = (int*)ws;
  int* kkh = bh + 2 * W;
  int* bv = kkh + (long)W * kh;
  int* kkv = bv + 2 * H;
  unsigned* tmp = (unsigned*)(kkv + (long)H * kv);
  resize_coeffs_kernel<<<cdiv(W, 64), 64, 0, st>>>(W0, W, kh, bh, kkh);
  resize_coeffs_kernel<<<cdiv(H, 64), 64, 0, st>>>(H0, H, kv, bv, kkv);
  // Pillow's horizontal pass only covers the source rows the vertical pass reads: [ybox_first, ybox_last).
  // Those bounds are a pure function of (H0, H); recompute them on the host the same way (double, no FMA).
  const double scale = (double)H0 / (double)H, support = scale < 1.0 ? 1.0 : scale;
  auto lo = [&](int yy) { int v = (int)((yy + 0.5) * scale - support + 0.5); return v < 0 ? 0 : v; };
  auto hi = [&](int yy) { int v = (int)((yy + 0.5) * scale + support + 0.5); return v > H0 ? H0 : v; };
  const int y0 = lo(0), y1 = hi(H - 1);
  const int rows = y1 - y0;
  const int F = B * T;
  // 2 source rows per workgroup (measured on MI355X at 1080p → 224²: 1 / 2 / 4 / 8 rows = 1.71 / 1.60 / 1.96 /
  // 2.92 ms per 512 frames: small LDS stages keep many workgroups per CU so staging and compute overlap)
  const int R = max(1, min(2, 16384 / W0));
  const int aligned = (W0 % 16 == 0) && (frame_stride % 16 == 0) && (((unsigned long)frames & 15) == 0);
  resize_h_kernel<<<dim3(cdiv(rows, R), F), 256, (size_t)R * W0 * 4, st>>>(frames, frame_stride, W0, frame_idx, y0,
                                                                           rows, R, W, kh, bh, kkh, tmp, aligned);
  resize_v_norm_kernel<<<dim3(cdiv((long)H * W, 256), F), 256, 0, st>>>(tmp, rows, y0, H, W, kv, bv, kkv, mean3[0],
                                                                         mean3[1], mean3[2], std3[0], std3[1], std3[2],
                                                                         T, channel_first, out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}

extern "C" long cmhar_imu_preprocess_ws(long total, int nrec, int C) { return total * C + 2L * nrec * C + 16; }

extern "C" int cmhar_imu_preprocess(int nrec, int C, const float* raw, const long* offsets, long total,
                                    const float* div_r, int median_k, int normalize, long nwin, const int* win_rec,
                                    const long* win_start, int win, float* out, float* ws, hipStream_t st) {
  if (nrec <= 0) return 0;
  if (C <= 0 || win <= 0 || median_k < 1 || median_k > 65 || median_k % 2 == 0) return -1;
  float* filt = ws;
  float* mean = ws + total * C;
  float* sd = mean + (long)nrec * C;
  imu_filter_stats_kernel<<<dim3(nrec, C), 256, 0, st>>>(raw, offsets, C, median_k, div_r, normalize, filt, mean,
                                                         sd);
  if (nwin > 0)
    imu_window_kernel<<<cdiv(nwin * C * win, 256), 256, 0, st>>>(filt, offsets, win_rec, win_start, C, win, mean,
                                                                  sd, nwin, out);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
