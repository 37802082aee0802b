// Probe (not product code): sustained int8 MFMA rate on RANDOM operands for
// the two int8 shapes, v_mfma_i32_32x32x32_i8 vs v_mfma_i32_16x16x64_i8, with
// independent accumulators (no back-to-back dependency: 4 chains of the
// 32x32 form, 8 chains of the 16x16 form), 8 waves per CU (two per SIMD, the
// product kernels' geometry), every CU busy, ~0.4 s per measurement so the
// chip sits at its loaded clock (MI355X_MICROARCH.md, DVFS give-back).
// Reports TOPS, the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) and
// the cycles per 32x32x32-equivalent MFMA per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_shape_probe.hip -o tools/probe/mfma_shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ __launch_bounds__(512, 1) void rate(const v4i* __restrict__ src, int iters, int* out,
                                               unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  v4i a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = src[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + i) * 64 + lane];
    b[i] = src[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + 8 + i) * 64 + lane];
  }
  v16i c[4] = {};
  v4i d[8] = {};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        c[i & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[(i + it) & 7], c[i & 3], 0, 0, 0);
    } else {  // 16 x 16x16x64 = the MACs of 8 x 32x32x32
#pragma unroll
      for (int i = 0; i < 16; ++i)
        d[i & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i & 7], b[(i + it + (i >> 3)) & 7], d[i & 7], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) s += c[0][g] + c[1][g] + c[2][g] + c[3][g];
#pragma unroll
  for (int k = 0; k < 8; ++k) s += d[k][0] + d[k][1] + d[k][2] + d[k][3];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  const int G = 256;  // one 8-wave workgroup per CU
  std::vector<int> h(G * 8 * 16 * 64 * 4);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (int)(x ^ (x >> 13));
  }
  v4i* src;
  int* out;
  unsigned long long* clk;
  if (hipMalloc(&src, h.size() * 4) || hipMalloc(&out, G * 512 * 4) || hipMalloc(&clk, G * 16) ||
      hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice))
    return 3;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 8000;
  for (int pass = 0; pass < 2; ++pass) {
    for (int kind = 0; kind < 2; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0, 0);
        for (int l = 0; l < 40; ++l) {
          if (kind == 0)
            hipLaunchKernelGGL(rate<0>, dim3(G), dim3(512), 0, 0, src, iters, out, clk);
          else
            hipLaunchKernelGGL(rate<1>, dim3(G), dim3(512), 0, 0, src, iters, out, clk);
        }
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 2;
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> c(G * 2);
        hipMemcpy(c.data(), clk, G * 16, hipMemcpyDeviceToHost);
        double ghz = 0, cyc = 0;
        for (int i = 0; i < G; ++i) {
          ghz += (double)c[2 * i] / (double)c[2 * i + 1] * 0.1;
          cyc += (double)c[2 * i];
        }
        ghz /= G;
        cyc /= G;
        // per SIMD: 2 waves x iters x 8 (32x32x32-equivalent MFMAs)
        const double per_mfma = cyc / (2.0 * iters * 8);
        const double ops = 40.0 * G * 8 /*waves*/ * iters * 8 /*32x32x32-equiv MFMAs*/ * 32768.0 * 2;
        printf("%s pass %d rep %d: %.1f ms  %.0f TOPS  clock %.3f GHz  %.2f cyc per 32x32x32-equiv per SIMD\n",
               kind == 0 ? "32x32x32_i8" : "16x16x64_i8", pass, rep, ms, ops / (ms * 1e-3) / 1e12, ghz, per_mfma);
      }
    }
  }
  return 0;
}
