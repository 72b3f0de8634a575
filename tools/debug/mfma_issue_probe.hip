// MFMA throughput with VALU work interleaved, per MFMA shape — does the attention's VALU density favour
// v_mfma_f32_32x32x16_bf16 or v_mfma_f32_16x16x32_bf16?  
//
// Every wave runs ITERS iterations of: 4 independent MFMA accumulation chains (of the 32x32x16 shape, or 8 chains of
// 16x16x32 — the same FLOPs per iteration), each MFMA followed by NV (32x32x16) or NV/2 (16x16x32) independent
// v_fma_f32, i.e. the same VALU work per FLOP for both shapes.  Launched at W waves per SIMD on every CU; the
// output is the chip's MFMA rate (dense bf16 TFLOP/s) and the VALU instructions per 32x32x16-equivalent.
//
// build: hipcc --offload-arch=gfx950 -O3 -o var/mfma_issue_probe tools/debug/mfma_issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define VALU(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(a), "v"(b))

template <int SHAPE, int NV>
__global__ __launch_bounds__(256) void probe(float* out, const bf16x8* __restrict__ ops, int iters, float a, float b) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  bf16x8 f[8];   // random operand fragments cycled through the chains (toggling data, as the library's peak probe)
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = ops[(tid * 8 + j) % 4096];
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = lane * 0.5f + j;
  float sink = 0.f;
  if constexpr (SHAPE == 0) {
    floatx16 c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = floatx16{};
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[q], f[q + 4], c[q], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < NV; ++v) VALU((q * NV + v) & 7);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) sink += c[q][r];
  } else {
    // inline asm with the accumulators pinned to AGPRs (the builtin form compiles to rotating register copies, as
    // in csrc/probe.hip)
    floatx4 c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {}, c7 = {};
#define M16(C, Q)                                                                                              \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(C) : "v"(f[Q]), "v"(f[((Q) + 3) & 7]));      \
  _Pragma("unroll") for (int v = 0; v < NV / 2 + ((NV & 1) && ((Q) & 1)); ++v) VALU(((Q) * NV + v) & 7);
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
      M16(c0, 0) M16(c1, 1) M16(c2, 2) M16(c3, 3) M16(c4, 4) M16(c5, 5) M16(c6, 6) M16(c7, 7)
    }
#undef M16
#pragma unroll
    for (int r = 0; r < 4; ++r) sink += c0[r] + c1[r] + c2[r] + c3[r] + c4[r] + c5[r] + c6[r] + c7[r];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sink += x[j];
  if (sink == 1234.5f) out[threadIdx.x] = sink;   // keeps everything live
}

template <int SHAPE, int NV>
static double run(int waves_per_simd, int iters, const bf16x8* ops) {
  float* out;
  hipMalloc(&out, 1024 * sizeof(float));
  const int blocks = 256 * waves_per_simd;   // 4 waves per block = one per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<SHAPE, NV><<<blocks, 256>>>(out, ops, iters / 8, 1.0001f, 0.5f);   // warm-up
  hipEventRecord(e0);
  probe<SHAPE, NV><<<blocks, 256>>>(out, ops, iters, 1.0001f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(out);
  const double flops = (double)blocks * 4 * iters * 4 * 32768.0;   // 4 x 32x32x16-equivalents per iteration
  return flops / (ms * 1e-3) / 1e12;
}

template <int NV>
static void row(int w, int iters, const bf16x8* ops) {
  const double t32 = run<0, NV>(w, iters, ops), t16 = run<1, NV>(w, iters, ops);
  printf("%d waves/SIMD  %2d VALU per 32x32x16-equivalent   32x32x16 %7.1f TF/s   16x16x32 %7.1f TF/s   ratio %.3f\n", w,
         NV, t32, t16, t16 / t32);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  // 4096 random bf16 fragments (values in [-1, 1))
  bf16x8 host[4096];
  unsigned s = 12345u;
  for (auto& v : host)
    for (int i = 0; i < 8; ++i) { s = s * 1664525u + 1013904223u; v[i] = (__bf16)((int)(s >> 9) * (1.f / 4194304.f) - 1.f); }
  bf16x8* ops;
  hipMalloc(&ops, sizeof(host));
  hipMemcpy(ops, host, sizeof(host), hipMemcpyHostToDevice);
  for (int w : {1, 2, 3}) {
    row<0>(w, iters, ops);
    row<2>(w, iters, ops);
    row<4>(w, iters, ops);
    row<6>(w, iters, ops);
    row<7>(w, iters, ops);
    row<8>(w, iters, ops);
    row<9>(w, iters, ops);
    row<10>(w, iters, ops);
    row<12>(w, iters, ops);
  }
  return 0;
}
