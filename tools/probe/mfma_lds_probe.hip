// Probe (not product code): one wave per SIMD, the block_l1 k-loop shape:
// per k-step 2 ds_read_b128 (prefetched 2 steps ahead) + 2 MFMA 32x32x32 i8,
// A operands rotating over 18 register fragments.  Variants: 0 = LDS reads,
// 1 = no LDS reads (B from registers), 2 = LDS reads with compiler-tracked loads.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <utility>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__device__ unsigned long long g_t[4096];

template <int OFF>
__device__ __forceinline__ v4i ds_read16(unsigned addr) {
  v4i r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void wait_lgkm_tie(v4i& x, v4i& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int V>
__global__ __launch_bounds__(256) void kloop(int iters, int* out) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += 256) ((v4i*)lds)[i] = v4i{i, i + 1, i + 2, i + 3};
  __syncthreads();
  v4i wr[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) wr[i] = v4i{i + lane, 3, 5, 7};
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  const unsigned a0 = base + 16 * lane, a1 = base + 16 * ((lane + 32) & 63) + 1024;
  v16i acc = {0};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    v16i c[2][2] = {{v16i{0}, v16i{0}}, {v16i{0}, v16i{0}}};
    v4i bf[3][2];
    auto ld = [&](auto nc, int buf) {
      constexpr int n = decltype(nc)::value;
      constexpr int off = 2048 * (n % 9) + (n & 1) * 32768;
      if constexpr (V == 2) {
        bf[buf][0] = *(const v4i*)(lds + (a0 - base) + off);
        bf[buf][1] = *(const v4i*)(lds + (a1 - base) + off);
      } else {
        bf[buf][0] = ds_read16<off>(a0);
        bf[buf][1] = ds_read16<off>(a1);
      }
    };
    if constexpr (V != 1) {
      ld(std::integral_constant<int, 0>{}, 0);
      ld(std::integral_constant<int, 1>{}, 1);
    }
    auto step = [&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      if constexpr (V == 1) {
        c[0][ks & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], wr[17 - ks], c[0][ks & 1], 0, 0, 0);
        c[1][ks & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], wr[(ks + 5) % 18], c[1][ks & 1], 0, 0, 0);
      } else {
        if constexpr (ks + 2 < 18) ld(std::integral_constant<int, ks + 2>{}, (ks + 2) % 3);
        constexpr int younger = (ks + 2 < 18 ? 2 : 0) + (ks + 1 < 18 ? 2 : 0);
        if constexpr (V == 0) wait_lgkm_tie<younger>(bf[ks % 3][0], bf[ks % 3][1]);
        c[0][ks & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], bf[ks % 3][0], c[0][ks & 1], 0, 0, 0);
        c[1][ks & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], bf[ks % 3][1], c[1][ks & 1], 0, 0, 0);
      }
    };
    static_for<0, 18>(step);
    acc += c[0][0] + c[0][1] + c[1][0] + c[1][1];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
  for (int g = 0; g < 16; ++g) s += acc[g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) g_t[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

int main() {
  int* out;
  hipMalloc(&out, 256 * 256 * 4);
  const int iters = 200;
  for (int v : {0, 1, 2}) {
    auto run = [&]() {
      if (v == 0) hipLaunchKernelGGL(kloop<0>, dim3(256), dim3(256), 0, 0, iters, out);
      if (v == 1) hipLaunchKernelGGL(kloop<1>, dim3(256), dim3(256), 0, 0, iters, out);
      if (v == 2) hipLaunchKernelGGL(kloop<2>, dim3(256), dim3(256), 0, 0, iters, out);
    };
    run();
    run();
    if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 2; }
    std::vector<unsigned long long> t(1024);
    hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_t), t.size() * 8);
    std::sort(t.begin(), t.end());
    printf("variant %d: %.1f ticks per MFMA (one wave per SIMD)\n", v, (double)t[512] / (iters * 36.0));
  }
  return 0;
}
