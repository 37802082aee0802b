// Probe (not product code): what one extra kernel boundary costs in a stream
// of dependent launches.  A "work" kernel (every CU busy ~T us) is launched
// back to back R times; then the same with an empty kernel, a one-workgroup
// kernel and a 256-workgroup small kernel between consecutive work launches.
// (time(with) - time(without)) / R = the cost of one extra launch boundary.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/launch_gap_probe.hip -o tools/probe/launch_gap_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(512) void work_kernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, 0.999f, b);
    b = __builtin_fmaf(b, 0.998f, a);
  }
  if (a == 12345.f) out[threadIdx.x] = b;  // never true; keeps the loop
}

__global__ void empty_kernel() {}

__global__ __launch_bounds__(256) void small_kernel(const int* __restrict__ x, int* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  y[i] = x[i] + 1;
}

int main() {
  float* out;
  int *x, *y;
  hipMalloc(&out, 4096);
  hipMalloc(&x, 1 << 20);
  hipMalloc(&y, 1 << 20);
  hipMemset(x, 0, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R = 50;
  for (int iters : {2000, 8000}) {
    float ms[4];
    for (int mode = 0; mode < 4; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {  // second repetition timed
        hipEventRecord(e0, 0);
        for (int r = 0; r < R; ++r) {
          hipLaunchKernelGGL(work_kernel, dim3(1024), dim3(512), 0, 0, out, iters);
          if (mode == 1) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0);
          if (mode == 2) hipLaunchKernelGGL(small_kernel, dim3(1), dim3(256), 0, 0, x, y);
          if (mode == 3) hipLaunchKernelGGL(small_kernel, dim3(256), dim3(256), 0, 0, x, y);
        }
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[mode], e0, e1);
      }
    }
    std::printf("work iters %d: %.2f us per work launch; extra boundary: empty %.2f us, 1-WG %.2f us, 256-WG %.2f us\n",
                iters, ms[0] * 1e3 / R, (ms[1] - ms[0]) * 1e3 / R, (ms[2] - ms[0]) * 1e3 / R,
                (ms[3] - ms[0]) * 1e3 / R);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
