// Probe (not product code): cycles per v_mfma_i32_32x32x32_i8 issued by one
// wave per SIMD with 1/2/4 independent accumulation chains, and with 2 waves
// per SIMD.  In-kernel s_memtime over the loop; median over waves.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__device__ unsigned long long g_t[4096];

template <int CH>
__global__ void chain(int iters, int* out, int seed) {
  v4i a = {seed + (int)threadIdx.x, seed * 3, 7, 11}, b = {5, seed, (int)threadIdx.x, 3};
  v16i c[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) c[i] = v16i{0};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8 / CH; ++r)
#pragma unroll
      for (int i = 0; i < CH; ++i) c[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c[i], 0, 0, 0);
    a = a + 1;  // keep operands live/changing
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i)
    for (int g = 0; g < 16; ++g) s += c[i][g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0 && blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64 < 4096)
    g_t[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
  int* out;
  hipMalloc(&out, 256 * 1024 * 4);
  const int iters = 2000;
  for (int waves : {4, 8}) {
    for (int ch : {1, 2, 4, 8}) {
      auto run = [&]() {
        dim3 g(256), blk(waves * 64);
        if (ch == 1) hipLaunchKernelGGL(chain<1>, g, blk, 0, 0, iters, out, 3);
        if (ch == 2) hipLaunchKernelGGL(chain<2>, g, blk, 0, 0, iters, out, 3);
        if (ch == 4) hipLaunchKernelGGL(chain<4>, g, blk, 0, 0, iters, out, 3);
        if (ch == 8) hipLaunchKernelGGL(chain<8>, g, blk, 0, 0, iters, out, 3);
      };
      run();
      run();
      if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 2; }
      std::vector<unsigned long long> t(256 * waves);
      hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_t), t.size() * 8);
      std::sort(t.begin(), t.end());
      const double per = (double)t[t.size() / 2] / (iters * 8.0);
      printf("waves/CU %d chains %d: %.1f memtime ticks per MFMA per wave (%.1f per MFMA per SIMD)\n", waves, ch, per,
             per * 4.0 / waves);
    }
  }
  return 0;
}
