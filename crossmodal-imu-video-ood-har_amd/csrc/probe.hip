// On-box MFMA peak probe ("peak = MI355X dense BF16 ≈ 2.5 PFLOP/s (vendor spec; confirm with an
// on-box MFMA microbenchmark and record it)").  Every wave issues back-to-back v_mfma_f32_32x32x16_bf16 on four
// independent accumulator chains whose operands cycle through eight random bf16 fragments (toggling data, as in a
// GEMM, not constant operands), so the matrix pipe of each SIMD stays full and the rate measured is the one the chip
// sustains at the clock it holds under dense MFMA load.  bench.py times one launch with HIP events and reports it as
// roofline.peak_measured beside the vendor figure.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void mfma_peak_kernel(int iters, const bf16x8* __restrict__ ops, int nops,
                                                        float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = ops[(tid * 8 + j) % nops];
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[0], f[1], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[2], f[3], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[4], f[5], c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[6], f[7], c3, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[1], f[4], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[3], f[6], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[5], f[0], c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[7], f[2], c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[tid] = s;     // keeps every chain live
}

}  // namespace

extern "C" long cmhar_mfma_peak_probe_flops(int blocks, int iters) {
  // per wave and iteration: 8 MFMAs of 2·32·32·16 FLOP; 4 waves per 256-thread workgroup
  return (long)blocks * 4 * iters * 8 * (2L * 32 * 32 * 16);
}

extern "C" int cmhar_mfma_peak_probe(int blocks, int iters, const void* ops, int nops, float* out,
                                     hipStream_t stream) {
  if (blocks <= 0 || iters <= 0 || nops <= 0 || !ops || !out) return -1;
  hipLaunchKernelGGL(mfma_peak_kernel, dim3(blocks), dim3(256), 0, stream, iters, (const bf16x8*)ops, nops, out);
  return (int)hipGetLastError();
}
