// Probe (not product code): latency of dependent global loads at kernel start,
// launched back to back (warm caches/TLB): s_memtime around (1) the first load
// of a buffer line, (2) the same line again, (3) another line 64 KiB away, (4) a
// line 64 MiB away, (5) 16 independent lines at once, (6) an LDS round trip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/lat_probe.hip -o tools/probe/lat_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void lat(const int* __restrict__ p, int* out, unsigned long long* st, int salt) {
  __shared__ int sh[64];
  unsigned long long t[8];
  int acc = 0;
  t[0] = __builtin_amdgcn_s_memtime();
  int v = __builtin_nontemporal_load(p + blockIdx.x * 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc += v;
  t[1] = __builtin_amdgcn_s_memtime();
  v = p[blockIdx.x * 16 + (acc & salt)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc += v;
  t[2] = __builtin_amdgcn_s_memtime();
  v = p[16384 + blockIdx.x * 16 + (acc & salt)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc += v;
  t[3] = __builtin_amdgcn_s_memtime();
  v = p[16 * 1024 * 1024 + blockIdx.x * 16 + (acc & salt)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc += v;
  t[4] = __builtin_amdgcn_s_memtime();
  int w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = p[4 * 1024 * 1024 + i * 65536 + blockIdx.x * 16 + (acc & salt)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += w[i];
  t[5] = __builtin_amdgcn_s_memtime();
  sh[threadIdx.x] = acc;
  __syncthreads();
  acc += sh[(threadIdx.x + 1) & 63];
  t[6] = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0)
    for (int i = 0; i < 6; ++i) st[blockIdx.x * 8 + i] = t[i + 1] - t[i];
}

int main() {
  int *p, *out;
  unsigned long long* st;
  const size_t n = 32u * 1024 * 1024;
  if (hipMalloc(&p, n * 4) || hipMalloc(&out, 256 * 64 * 4) || hipMalloc(&st, 256 * 64)) return 3;
  hipMemset(p, 0, n * 4);
  const char* nm[6] = {"first load (nt)", "same line again", "line +64KiB", "line +64MiB", "16 lines at once", "LDS+barrier"};
  for (int G : {1, 256}) {
    for (int it = 0; it < 50; ++it) hipLaunchKernelGGL(lat, dim3(G), dim3(64), 0, 0, p, out, st, 0);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(G * 8);
    hipMemcpy(h.data(), st, G * 64, hipMemcpyDeviceToHost);
    printf("grid %d (median over workgroups, s_memtime cycles):\n", G);
    for (int k = 0; k < 6; ++k) {
      std::vector<unsigned long long> d;
      for (int b = 0; b < G; ++b) d.push_back(h[b * 8 + k]);
      std::sort(d.begin(), d.end());
      printf("  %-18s %llu\n", nm[k], d[d.size() / 2]);
    }
  }
  return 0;
}
