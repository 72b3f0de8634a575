// Diagnostic: are 256 one-per-CU workgroups (160 KiB LDS each) co-resident on the MI355X?  Each workgroup records
// its XCC id, hardware CU id (HW_REG_HW_ID) and start/end timestamps, spinning ~50 us.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ __launch_bounds__(512) void probe(unsigned* info, long long* t) {
  __shared__ char smem[163840];
  if (threadIdx.x == 0) {
    unsigned xcc, hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    long long t0 = wall_clock64();
    smem[0] = 1;
    while (wall_clock64() - t0 < 5000) __builtin_amdgcn_s_sleep(10);   // ~50 us at 100 MHz
    info[2 * blockIdx.x] = xcc;
    info[2 * blockIdx.x + 1] = hwid;
    t[2 * blockIdx.x] = t0;
    t[2 * blockIdx.x + 1] = wall_clock64();
  }
  __syncthreads();
  if (smem[0] == 2) info[0] = 0;
}
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("CUs %d, LDS/block %zu, wall clock %d kHz\n", p.multiProcessorCount, p.sharedMemPerBlock, p.clockRate);
  const int n = 256;
  unsigned* info; long long* t;
  hipMalloc(&info, 8 * n); hipMalloc(&t, 16 * n);
  for (int rep = 0; rep < 2; ++rep) probe<<<n, 512>>>(info, t);
  hipDeviceSynchronize();
  unsigned hi[2 * n]; long long ht[2 * n];
  hipMemcpy(hi, info, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(ht, t, 16 * n, hipMemcpyDeviceToHost);
  long long mn = ht[0], mx = ht[0];
  int late = 0;
  for (int i = 0; i < n; ++i) { if (ht[2 * i] < mn) mn = ht[2 * i]; }
  for (int i = 0; i < n; ++i) { if (ht[2 * i] - mn > 2500) ++late; if (ht[2*i] > mx) mx = ht[2*i]; }
  int per_xcc[8] = {0};
  for (int i = 0; i < n; ++i) per_xcc[hi[2 * i] & 7]++;
  printf("start spread %lld ticks, workgroups starting > half a spin late: %d\n", mx - mn, late);
  for (int x = 0; x < 8; ++x) printf("xcc %d: %d wgs\n", x, per_xcc[x]);
  for (int i = 0; i < 16; ++i) printf("wg %d xcc %u hwid 0x%08x start %lld\n", i, hi[2*i], hi[2*i+1], ht[2*i] - mn);
  return 0;
}
