// Ablation build of the ping-pong GEMM (NOT part of the product library).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I include tools/debug/gemm_pp_ablate.hip -o tools/debug/libablate_pp.so
#include "gemm_pp.hip"

extern "C" int ablate_pp(int mode, int act, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                         void* C, long ldc, void* aux, void* stamps, int delay, hipStream_t st) {
  Epilogue e{};
  e.alpha = 1.f;
  e.act = act;
  e.aux_out = aux;
  e.ldo = N;
  e.rowsum = (float*)stamps;
  const int units = (M / PM) * (N / PN);
  int G = 512;
  if (units < G) G = ((units + 7) / 8) * 8;
  int gn = 1;
  while (gn < 8 && (long)N / gn * K * 2 > (2l << 20) && (N / PN) % (gn * 2) == 0) gn *= 2;
#define G_(MD, AC) gemm_pp_kernel<true, true, bf16, AC, MD><<<G, PT, 0, st>>>(M, N, K, (const bf16*)A, lda, \
    (const bf16*)B, ldb, (bf16*)C, ldc, e, K, 1, 0, delay, gn)
  if (act == ACT_GELU_SAVEGRAD) {
    if (mode == 0) G_(0, ACT_GELU_SAVEGRAD); else if (mode == 1) G_(1, ACT_GELU_SAVEGRAD);
    else if (mode == 3) G_(3, ACT_GELU_SAVEGRAD); else G_(4, ACT_GELU_SAVEGRAD);
  } else {
    if (mode == 0) G_(0, ACT_NONE); else if (mode == 1) G_(1, ACT_NONE); else if (mode == 3) G_(3, ACT_NONE);
    else G_(4, ACT_NONE);
  }
  return (int)hipGetLastError();
}
