// Probe (not product code): LDS throughput of the access patterns the stem
// could use, 8 waves x 2 workgroups per CU on every CU: ds_read_b64 with the
// lanes' 8-byte windows 2 bytes apart (unaligned: start 2*lane + 5), the same
// 8-byte-aligned (4 shifted copies), and ds_write_b16 at odd vs even byte
// addresses.  Reports LDS cycles per wave-instruction (s_memtime per CU).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/lds_tput_probe.hip -o tools/probe/lds_tput_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(512) void tp(unsigned* sink, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[32768];
  for (int i = threadIdx.x; i < 32768 / 4; i += 512) ((unsigned*)lds)[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5, w = threadIdx.x >> 6;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
  unsigned a;
  if (MODE == 0) a = base + 2 * lr + 5 + lh * 3200 + w * 800;          // unaligned b64 (stem octet read)
  else if (MODE == 1) a = base + ((2 * lr + 5 + 7) & ~7) + (lr & 3) * 1024 + lh * 3200 + w * 800;  // aligned copies
  else if (MODE == 2) a = base + 2 * lane + 1 + w * 256;                // odd b16 writes
  else a = base + 2 * lane + w * 256;                                   // even b16 writes
  unsigned acc = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 256; ++it) {
    if constexpr (MODE < 2) {
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
      v2u v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[k]) : "v"(a), "n"(k * 256) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k][0] ^ v[k][1];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("ds_write_b16 %0, %1 offset:%2" ::"v"(a), "v"(acc + k), "n"(k * 2048) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 512 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  unsigned* sink;
  unsigned long long* cyc;
  if (hipMalloc(&sink, 512 * 512 * 4) || hipMalloc(&cyc, 512 * 8)) return 3;
  const char* nm[4] = {"ds_read_b64 unaligned (2*lane+5)", "ds_read_b64 aligned (4 copies)", "ds_write_b16 odd bytes",
                       "ds_write_b16 even bytes"};
  for (int m = 0; m < 4; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      if (m == 0) hipLaunchKernelGGL(tp<0>, dim3(512), dim3(512), 0, 0, sink, cyc);
      if (m == 1) hipLaunchKernelGGL(tp<1>, dim3(512), dim3(512), 0, 0, sink, cyc);
      if (m == 2) hipLaunchKernelGGL(tp<2>, dim3(512), dim3(512), 0, 0, sink, cyc);
      if (m == 3) hipLaunchKernelGGL(tp<3>, dim3(512), dim3(512), 0, 0, sink, cyc);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // per CU: 2 workgroups x 8 waves x 256 x 8 instructions
    printf("%-36s %.2f cycles per wave-instruction per CU\n", nm[m], (double)c / (2.0 * 8 * 256 * 8));
  }
  return 0;
}
