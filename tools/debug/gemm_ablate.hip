// Ablation build of the 256² GEMM (NOT part of the product library): times DMA-only / MFMA-only variants.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I include tools/debug/gemm_ablate.hip -o tools/debug/libablate.so
#include "../../crossmodal-imu-video-ood-har_amd/csrc/gemm_bf16.hip"
namespace {
#include "gemm256p.inc"
}

extern "C" int ablate_gemm256(int mode, int layout, int M, int N, int K, const void* A, long lda, const void* B,
                              long ldb, void* C, long ldc, hipStream_t st) {
  Epilogue e{};
  e.alpha = 1.f;
  dim3 grid((M / TM2) * (N / TN2), 1, 1);
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  bf16* c = (bf16*)C;
#define G(AK, BK, MD) gemm256_kernel<AK, BK, bf16, MD><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0, nullptr, 0, 0)
#define L3(AK, BK) if (mode == 0) G(AK, BK, 0); \
  else if (mode == 3) G(AK, BK, 3); else if (mode == 4) G(AK, BK, 4); \
  else if (mode == 5) G(AK, BK, 5); else if (mode == 7) G(AK, BK, 7); else if (mode == 8) G(AK, BK, 8); \
  else if (mode == 9) gemm256_kernel<AK, BK, bf16, 0, 3><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, \
                                                                           0, nullptr, 0, 0); \
  else if (mode == 10) gemm256_kernel<AK, BK, bf16, 4, 3><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, \
                                                                            0, 0, nullptr, 0, 0); \
  else G(AK, BK, 6);
  if (layout == 0) { L3(true, true) } else if (layout == 1) { L3(true, false) } else { L3(false, false) }
  return (int)hipGetLastError();
}

extern "C" int ablate_gemm128(int layout, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                              void* C, long ldc, hipStream_t st) {
  Epilogue e{};
  e.alpha = 1.f;
  dim3 grid((M / BM) * (N / BN), 1, 1);
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  bf16* c = (bf16*)C;
  if (layout == 0) gemm_bf16_kernel<true, true, bf16, false><<<grid, NT, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  else if (layout == 1) gemm_bf16_kernel<true, false, bf16, false><<<grid, NT, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  else gemm_bf16_kernel<false, false, bf16, false><<<grid, NT, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  return (int)hipGetLastError();
}

extern "C" int ablate_gemm256p(int layout, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                               void* C, long ldc, hipStream_t st) {
  Epilogue e{};
  e.alpha = 1.f;
  dim3 grid((M / TM2) * (N / TN2), 1, 1);
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  bf16* c = (bf16*)C;
  if (layout == 0) gemm256p_kernel<true, true, bf16><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  else if (layout == 1) gemm256p_kernel<true, false, bf16><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  else gemm256p_kernel<false, false, bf16><<<grid, NT2, 0, st>>>(M, N, K, a, lda, b, ldb, c, ldc, e, K, 0, 0);
  return (int)hipGetLastError();
}
