// Probe (not product code): per-CU throughput of LDS-DMA (global_load_lds_dwordx4)
// vs register loads (global_load_dwordx4) on gfx950, for L2-resident and
// shared (every CU reads the same bytes) sources.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/ldsdma_bw.hip -o tools/probe/ldsdma_bw
// Run:   ./ldsdma_bw <mode 0=lds-dma 1=vgpr> <KiB per CU region> <shared 0/1> <waves 4/8> <depth>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void bw_kernel(const int8_t* src, int region, int shared, int iters, int depth,
                                                    int nwaves, int* sink) {
  __shared__ __attribute__((aligned(16))) int8_t lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= nwaves) return;
  const int8_t* base = src + (shared ? 0 : (size_t)blockIdx.x * region);
  const int npieces = region / 1024;
  v4i acc = {0, 0, 0, 0};
  int pc = wave;
  for (int it = 0; it < iters; ++it) {
    for (int d = 0; d < 8; ++d) {
      const int8_t* g = base + (size_t)(pc % npieces) * 1024 + lane * 16;
      if constexpr (MODE == 0) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(lds + ((wave * 8 + d) & 127) * 1024),
                                         16, 0, 0);
      } else {
        acc += *(const v4i*)g;
      }
      pc += nwaves;
    }
    if (depth <= 8)
      __builtin_amdgcn_s_waitcnt(0x0070 | 0);
    else
      __builtin_amdgcn_s_waitcnt(0x0070 | 8);
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  if (acc[0] == 0x12345678) sink[0] = acc[1] + lds[lane];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int kib = argc > 2 ? atoi(argv[2]) : 64;
  const int shared = argc > 3 ? atoi(argv[3]) : 0;
  const int nwaves = argc > 4 ? atoi(argv[4]) : 8;
  const int depth = argc > 5 ? atoi(argv[5]) : 16;
  const int region = kib * 1024, iters = 400;
  int8_t* src;
  int* sink;
  hipMalloc(&src, (size_t)256 * region);
  hipMemset(src, 1, (size_t)256 * region);
  hipMalloc(&sink, 64);
  auto run = [&]() {
    if (mode == 0)
      hipLaunchKernelGGL(bw_kernel<0>, dim3(256), dim3(512), 0, 0, src, region, shared, iters, depth, nwaves, sink);
    else
      hipLaunchKernelGGL(bw_kernel<1>, dim3(256), dim3(512), 0, 0, src, region, shared, iters, depth, nwaves, sink);
  };
  run();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  run();
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = 256.0 * nwaves * iters * 8 * 1024;
  printf("mode=%s region=%dKiB shared=%d waves=%d depth=%d: %.1f us, %.1f GB/s per CU, %.2f TB/s chip\n",
         mode ? "vgpr" : "ldsdma", kib, shared, nwaves, depth, ms * 1e3, bytes / 256 / (ms * 1e-3) / 1e9,
         bytes / (ms * 1e-3) / 1e12);
  return 0;
}
