// Energy-score OOD head (BASELINE config 5 / SURVEY §8(f) rank 1).  The reference has no OOD code: the
// logits come from the reference's prediction path (`Evaluator.predict`, src/eval/evaluator.py:28-53, which takes
// `logits.max(1)`), and the score is the energy E = −T·logsumexp(logits / T) (lower energy = more in-distribution).
//
// One pass over the logits: per row, the prediction (first index of the maximum — torch.max's CPU tie rule), the
// maximum logit and the energy.  One wave per row, lanes striding over the classes; wave reductions by cross-lane
// shuffles.  HBM-bound (N·C·dtype bytes read once).
#include "common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void logits_energy_kernel(int N, int C, const T* __restrict__ L, long ld,
                                                            float inv_t, float t, int* __restrict__ pred,
                                                            float* __restrict__ energy, float* __restrict__ maxv) {
  const int row = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;                                   // wave-uniform
  const T* r = L + (long)row * ld;
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int j = lane; j < C; j += 64) {
    const float v = to_f<T>(r[j]);
    if (v > m) { m = v; am = j; }                         // strict: the first maximum of this lane's columns
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float mo = __shfl_xor(m, off);
    const int ao = __shfl_xor(am, off);
    if (mo > m || (mo == m && ao < am)) { m = mo; am = ao; }
  }
  float s = 0.f;
  for (int j = lane; j < C; j += 64) s += __expf((to_f<T>(r[j]) - m) * inv_t);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) {
    if (pred) pred[row] = am;
    if (maxv) maxv[row] = m;
    if (energy) energy[row] = -t * (m * inv_t + __logf(s));
  }
}

}  // namespace

extern "C" int cmhar_logits_energy(int dtype, int N, int C, const void* logits, long ld, float temperature, int* pred,
                                   float* energy, float* maxlogit, hipStream_t st) {
  if (N <= 0) return 0;
  if (C <= 0 || ld < C || !(temperature > 0.f)) return -1;
  const int blocks = cdiv((long)N * 64, 256);
  if (dtype == CMHAR_BF16)
    logits_energy_kernel<bf16><<<blocks, 256, 0, st>>>(N, C, (const bf16*)logits, ld, 1.f / temperature, temperature,
                                                       pred, energy, maxlogit);
  else
    logits_energy_kernel<float><<<blocks, 256, 0, st>>>(N, C, (const float*)logits, ld, 1.f / temperature,
                                                        temperature, pred, energy, maxlogit);
  CMHAR_CHECK_LAUNCH();
  return 0;
}
