// On-box MFMA peak probe ("peak = MI355X dense BF16 ≈ 2.5 PFLOP/s (vendor spec; confirm with an
// on-box MFMA microbenchmark and record it)").  Every wave issues back-to-back bf16 MFMAs on eight independent
// accumulator chains whose operands cycle through eight random bf16 fragments (toggling data, as in a GEMM, not
// constant operands), so the matrix pipe of each SIMD stays full and the rate measured is the one the chip sustains
// at the clock it holds under dense MFMA load.  Two shapes: v_mfma_f32_32x32x16_bf16 (shape 0, the flash-attention
// kernels) and v_mfma_f32_16x16x32_bf16 (shape 1, the GEMMs) — on random data the chip holds a different clock for
// each (MI355X_MICROARCH.md, DVFS item 7).  bench.py times one launch of each with HIP events and reports the larger
// as roofline.peak_measured beside the vendor figure.
#include "common.h"

namespace {

template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_peak_kernel(int iters, const bf16x8* __restrict__ ops, int nops,
                                                        float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = ops[(tid * 8 + j) % nops];
  float s = 0.f;
  if constexpr (SHAPE == 0) {
    floatx16 c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = floatx16{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[k], f[(k + 3) & 7], c[k], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += c[k][r];
  } else {
    // issued by inline asm with the accumulators pinned to AGPRs: the builtin form compiled to a rotating register
    // assignment with 12 v_accvgpr_mov per 8 MFMAs (measured, probe.s); eight chains keep every dependent pair 7
    // MFMAs apart, beyond any MFMA dependency hazard window
    floatx4 c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {}, c7 = {};
#define MF16(C, A, B) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(C) : "v"(A), "v"(B))
    for (int it = 0; it < iters; ++it) {
      MF16(c0, f[0], f[3]);
      MF16(c1, f[1], f[4]);
      MF16(c2, f[2], f[5]);
      MF16(c3, f[3], f[6]);
      MF16(c4, f[4], f[7]);
      MF16(c5, f[5], f[0]);
      MF16(c6, f[6], f[1]);
      MF16(c7, f[7], f[2]);
    }
#undef MF16
#pragma unroll
    for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r] + c4[r] + c5[r] + c6[r] + c7[r];
  }
  out[tid] = s;     // keeps every chain live
}

}  // namespace

extern "C" long cmhar_mfma_peak_probe_flops(int shape, int blocks, int iters) {
  // per wave and iteration: 8 MFMAs of 2·32·32·16 (shape 0) or 2·16·16·32 (shape 1) FLOP; 4 waves per workgroup
  const long per = shape == 0 ? 2L * 32 * 32 * 16 : 2L * 16 * 16 * 32;
  return (long)blocks * 4 * iters * 8 * per;
}

extern "C" int cmhar_mfma_peak_probe(int shape, int blocks, int iters, const void* ops, int nops, float* out,
                                     hipStream_t stream) {
  if (blocks <= 0 || iters <= 0 || nops <= 0 || !ops || !out || shape < 0 || shape > 1) return -1;
  if (shape == 0)
    hipLaunchKernelGGL(mfma_peak_kernel<0>, dim3(blocks), dim3(256), 0, stream, iters, (const bf16x8*)ops, nops, out);
  else
    hipLaunchKernelGGL(mfma_peak_kernel<1>, dim3(blocks), dim3(256), 0, stream, iters, (const bf16x8*)ops, nops, out);
  return (int)hipGetLastError();
}
