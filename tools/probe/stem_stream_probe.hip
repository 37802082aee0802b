// Probe (not product code): HBM read rate of the stem's input access pattern
// alone (fp32 NCHW [256][3][224][224], 154 MB): 512 bands of 28 pooled rows =
// 116 input rows x 3 planes, two 512-thread workgroups per CU; variants:
// (0) float2 per lane, 64 lanes = 512 B of one row (the stem's loads),
// (1) float4 per lane, (2) float4 per lane with 8 rows in flight per thread.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/stem_stream_probe.hip -o tools/probe/stem_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(512, 2) void stream(const float* __restrict__ x, int N, float* out) {
  const int tid = threadIdx.x;
  float acc = 0.f;
  for (int item = blockIdx.x; item < N * 2; item += gridDim.x) {
    const int n = item >> 1, band = item & 1;
    const float* img = x + (size_t)n * 3 * 224 * 224;
    const int r0 = band * 112, r1 = r0 + 112;
    if constexpr (MODE == 0) {  // per step: 4 rows x 112 float2 x 3 planes (the stem)
      const int r = tid >> 7, u = tid & 127;
      for (int row = r0; row < r1; row += 4) {
        if (u < 112) {
          const float* src = img + (size_t)(row + r) * 224 + 2 * u;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const float2 v = *(const float2*)(src + (size_t)c * 224 * 224);
            acc += v.x + v.y;
          }
        }
      }
    } else {  // float4 per lane: 8 rows x 56 float4 per step
      const int r = tid >> 6, u = tid & 63;
      for (int row = r0; row < r1; row += (MODE == 1 ? 8 : 16)) {
        if (u < 56) {
#pragma unroll
          for (int h = 0; h < (MODE == 1 ? 1 : 2); ++h) {
            const float* src = img + (size_t)(row + r + 8 * h) * 224 + 4 * u;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const float4 v = *(const float4*)(src + (size_t)c * 224 * 224);
              acc += v.x + v.y + v.z + v.w;
            }
          }
        }
      }
    }
  }
  out[blockIdx.x * 512 + tid] = acc;
}

int main() {
  const int N = 256;
  float *x, *out;
  const size_t nx = (size_t)N * 3 * 224 * 224;
  if (hipMalloc(&x, nx * 4) || hipMalloc(&out, 512 * 512 * 4)) return 3;
  hipMemset(x, 0, nx * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e9;
    for (int rep = 0; rep < 10; ++rep) {
      hipEventRecord(e0, 0);
      if (mode == 0) hipLaunchKernelGGL(stream<0>, dim3(512), dim3(512), 0, 0, x, N, out);
      if (mode == 1) hipLaunchKernelGGL(stream<1>, dim3(512), dim3(512), 0, 0, x, N, out);
      if (mode == 2) hipLaunchKernelGGL(stream<2>, dim3(512), dim3(512), 0, 0, x, N, out);
      hipEventRecord(e1, 0);
      if (hipEventSynchronize(e1) != hipSuccess) return 2;
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("mode %d: %.1f us  %.2f TB/s\n", mode, best * 1e3, nx * 4 / (best * 1e-3) / 1e12);
  }
  return 0;
}
