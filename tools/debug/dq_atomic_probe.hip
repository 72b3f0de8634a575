// Probe (round 6): what fp32 atomic accumulation of the flash backward's dQ would cost if the dK/dV kernel produced
// dQ itself (FA2-style: each 128-key workgroup adds its 64-query x 64-dim dQ partial per query tile into an fp32
// dQ accumulator), against the dQ kernel's ~360 us per layer at B*H = 384, L = 1568, D = 64.
// Traffic shape: 384 heads x 13 key blocks x 25 query tiles x 4096 floats = 2.0 GB of no-return float atomics per
// layer; each wave adds a 16-row x 64-dim slice (16 floats per lane, one row-contiguous 256-B line per instruction).
// Variants: 0 = atomics (agent scope, relaxed), 1 = plain stores of the same bytes to a private slab (the
// non-atomic write rate for comparison).  Build: hipcc --offload-arch=gfx950 -O3 dq_atomic_probe.hip -o /tmp/dqp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int BH = 384, L = 1568, D = 64, KB = 13, QT = (L + 63) / 64;

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* __restrict__ acc, float* __restrict__ slab, float v) {
  const int bh = blockIdx.x / KB, kb = blockIdx.x % KB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = qt * 64 + wave * 16 + r;
      if (q >= L) break;
      const long idx = ((long)bh * L + q) * D + lane;
      if (MODE == 0) {
        __hip_atomic_fetch_add(acc + idx, v * (float)(kb + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        slab[(long)kb * BH * L * D + idx] = v * (float)(kb + 1);
      }
    }
  }
}

int main() {
  const long n = (long)BH * L * D;
  float *acc, *slab;
  if (hipMalloc(&acc, n * 4) != hipSuccess || hipMalloc(&slab, n * 4 * KB) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 4; ++rep) {
      hipMemset(acc, 0, n * 4);
      hipEventRecord(e0);
      if (mode == 0) probe<0><<<BH * KB, 256>>>(acc, slab, 1.f);
      else probe<1><<<BH * KB, 256>>>(acc, slab, 1.f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double bytes = (double)n * KB * 4;
      printf("%s rep %d: %.1f us, %.2f TB/s of added floats\n", mode == 0 ? "atomic add" : "plain store", rep,
             ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
  }
  // check: every element of acc = sum_{kb} (kb+1) = KB(KB+1)/2
  std::vector<float> h(4096);
  hipMemset(acc, 0, n * 4);
  probe<0><<<BH * KB, 256>>>(acc, slab, 1.f);
  hipMemcpy(h.data(), acc + n - 4096, 4096 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (float x : h) bad += x != (float)(KB * (KB + 1) / 2);
  printf("check: %d bad of 4096\n", bad);
  hipFree(acc);
  hipFree(slab);
  return bad != 0;
}
