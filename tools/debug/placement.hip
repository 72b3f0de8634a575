// Where do the workgroups of a 512-block, 72 KiB-LDS, 256-thread launch land?  Records per block the hardware ids
// (XCC_ID, HW_ID: cu/sh/se/tg) of wave 0.   hipcc --offload-arch=gfx950 -O3 tools/debug/placement.hip -o /tmp/placement
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <map>
#include <vector>

__global__ __launch_bounds__(256, 2) void probe(unsigned* out, int spin) {
  __shared__ char smem[73728];
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));     // HW_REG_HW_ID, offset 0, size 32
    unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    smem[0] = 1;
  }
  const long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < spin) __builtin_amdgcn_s_sleep(8);
  if (smem[0] == 7) out[0] = 0;
}

int main() {
  const int G = 512;
  unsigned* d;
  if (hipMalloc(&d, G * 2 * sizeof(unsigned)) != hipSuccess) return 1;
  probe<<<G, 256>>>(d, 2000000);
  std::vector<unsigned> h(G * 2);
  if (hipMemcpy(h.data(), d, G * 2 * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::map<unsigned, std::vector<int>> cu;
  for (int b = 0; b < G; ++b) {
    unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    unsigned cu_id = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7, tg = (hw >> 16) & 0xf;
    unsigned key = (xcc << 12) | (se << 8) | (sh << 4) | cu_id;
    cu[key].push_back(b);
    if (b < 24 || (b >= 256 && b < 264)) printf("block %3d xcc %u se %u sh %u cu %2u tg %u\n", b, xcc, se, sh, cu_id, tg);
  }
  int pairs_256 = 0, total = 0;
  std::map<int, int> diff;
  for (auto& kv : cu) {
    total++;
    if (kv.second.size() == 2) diff[kv.second[1] - kv.second[0]]++;
    else printf("cu %x hosts %zu blocks\n", kv.first, kv.second.size());
  }
  printf("distinct CUs %d\n", total);
  for (auto& kv : diff) printf("pair block distance %d: %d CUs\n", kv.first, kv.second);
  return 0;
}
