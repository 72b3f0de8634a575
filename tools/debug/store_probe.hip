// Store-issue probe: per-CU rate of 16-B-per-lane global stores by how many bytes of one row an instruction covers.
// One 512-thread workgroup per CU (grid = NWG <= 256), each writing a 256x256 bf16 tile (128 KiB, row pitch P bytes)
// REPS times, as the GEMM epilogue does.  Mode = bytes of one row covered by one wave instruction: 64 (the persistent
// GEMM's register-direct epilogue: 16 rows x 64 B), 128 (8 rows x 128 B), 256 (4 x 256), 512 (2 x 512).
// Prints cycles per tile (s_memtime, per workgroup averaged) and B/clk per CU.
// build: hipcc --offload-arch=gfx950 -O3 -o store_probe tools/debug/store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int RB, int SW, int VALU>
__global__ __launch_bounds__(512) void probe(char* __restrict__ out, long pitch, int reps, int nt,
                                             unsigned long long* __restrict__ cyc) {
  constexpr int LPR = RB / 16;          // lanes per row
  constexpr int RPI = 64 / LPR;         // rows per instruction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* tile = out + (long)blockIdx.x * 256 * pitch;
  const u32x4 v = {(unsigned)lane, (unsigned)wave, 1u, 2u};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    // the tile: 256 rows x 512 B; column block cb of RB bytes, row group; wave w takes 1/8 of the instructions
    constexpr int NI = 256 * 512 / 1024;   // 128 instructions of 1 KiB per tile
#pragma unroll 4
    for (int i = wave; i < NI; i += SW) {
      if (wave >= SW) break;
      const int cb = i % (512 / RB), rg = i / (512 / RB);
      const int row = rg * RPI + lane / LPR, col = cb * RB + (lane % LPR) * 16;
      u32x4 w = v;
      w.z = (unsigned)(r + i);
      // VALU between stores (the epilogue's swaps / converts): a dependent chain of VALU adds
#pragma unroll
      for (int k = 0; k < VALU; ++k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(w.x) : "v"(w.y));
      if (nt)
        __builtin_nontemporal_store(w, (u32x4*)(tile + (long)row * pitch + col));
      else
        *(u32x4*)(tile + (long)row * pitch + col) = w;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int RB, int SW = 8, int VALU = 0>
void run(char* out, long pitch, int nwg, int reps, int nt, unsigned long long* cyc) {
  hipLaunchKernelGGL((probe<RB, SW, VALU>), dim3(nwg), dim3(512), 0, 0, out, pitch, reps, nt, cyc);   // warm
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<RB, SW, VALU>), dim3(nwg), dim3(512), 0, 0, out, pitch, reps, nt, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(nwg);
  hipMemcpy(h.data(), cyc, nwg * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto c : h) avg += (double)c;
  avg /= nwg;
  const double bytes = 131072.0 * reps;
  // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH constants table)
  printf("storing waves %d valu/store %2d rowbytes %4d nt %d wgs %3d: %8.0f clk/tile  %6.2f B/clk/CU  event %.3f ms  chip %.2f TB/s\n", SW, VALU, RB, nt, nwg,
         avg / reps, bytes / avg, ms, bytes * nwg / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
  const long pitch = argc > 1 ? atol(argv[1]) : 4608;
  const int reps = 8;
  char* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256L * 256 * pitch + 4096);
  hipMalloc(&cyc, 256 * 8);
  for (int nwg : {32, 256})
    for (int nt : {0, 1}) {
      run<64>(out, pitch, nwg, reps, nt, cyc);
      run<128>(out, pitch, nwg, reps, nt, cyc);
      run<256>(out, pitch, nwg, reps, nt, cyc);
      run<512>(out, pitch, nwg, reps, nt, cyc);
    }
  for (int nwg : {32, 256}) {
    run<64, 4, 0>(out, pitch, nwg, reps, 1, cyc);
    run<64, 4, 16>(out, pitch, nwg, reps, 1, cyc);
    run<64, 8, 16>(out, pitch, nwg, reps, 1, cyc);
    run<64, 2, 0>(out, pitch, nwg, reps, 1, cyc);
    run<64, 1, 0>(out, pitch, nwg, reps, 1, cyc);
    run<128, 4, 16>(out, pitch, nwg, reps, 1, cyc);
  }
  hipFree(out);
  hipFree(cyc);
  return 0;
}
