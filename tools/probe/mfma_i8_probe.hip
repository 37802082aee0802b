// Probe: int8 MFMA operand/accumulator layouts and issue rate on gfx950.
// Verifies the lane maps the conv kernels rely on, and measures ops/clk for
// v_mfma_i32_32x32x32_i8, v_mfma_i32_16x16x64_i8 and v_mfma_i32_32x32x16_i8.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <chrono>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while(0)

// A: [32][32] int8 row-major (row i, k), B: [32][32] int8 stored as [col j][k]; D: [32][32] int32 [i][j]
__global__ void k32x32x32(const int8_t* A, const int8_t* Bt, int* D) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  v4i a = *(const v4i*)(A + r * 32 + 16 * h);
  v4i b = *(const v4i*)(Bt + r * 32 + 16 * h);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int g = 0; g < 16; ++g) {
    int row = (g & 3) + 8 * (g >> 2) + 4 * h;
    D[row * 32 + r] = c[g];
  }
}
__global__ void k16x16x64(const int8_t* A, const int8_t* Bt, int* D) {
  int l = threadIdx.x, r = l & 15, q = l >> 4;
  v4i a = *(const v4i*)(A + r * 64 + 16 * q);
  v4i b = *(const v4i*)(Bt + r * 64 + 16 * q);
  v4i c = {0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int g = 0; g < 4; ++g) D[(4 * q + g) * 16 + r] = c[g];
}
__global__ void k32x32x16(const int8_t* A, const int8_t* Bt, int* D) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  long a = *(const long*)(A + r * 16 + 8 * h);
  long b = *(const long*)(Bt + r * 16 + 8 * h);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x16_i8(a, b, c, 0, 0, 0);
  for (int g = 0; g < 16; ++g) {
    int row = (g & 3) + 8 * (g >> 2) + 4 * h;
    D[row * 32 + r] = c[g];
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void rate(int iters, int* out, int seed) {
  v4i a = {seed + (int)threadIdx.x, seed * 3, 7, 11}, b = {5, seed, (int)threadIdx.x, 3};
  long a8 = a[0], b8 = b[1];
  v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  v4i d0 = {0}, d1 = {0}, d2 = {0}, d3 = {0};
  for (int i = 0; i < iters; ++i) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
    } else if constexpr (KIND == 1) {
      d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, d3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_i32_32x32x16_i8(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x16_i8(b8, a8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_32x32x16_i8(a8, a8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_32x32x16_i8(b8, b8, c3, 0, 0, 0);
    }
  }
  int s = 0;
  for (int g = 0; g < 16; ++g) s += c0[g] + c1[g] + c2[g] + c3[g];
  for (int g = 0; g < 4; ++g) s += d0[g] + d1[g] + d2[g] + d3[g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static int check(const char* name, int M, int N, int K, void (*kern)(const int8_t*, const int8_t*, int*)) {
  std::vector<int8_t> A(M * K), B(N * K);
  srand(1234);
  for (auto& v : A) v = (int8_t)(rand() % 255 - 127);
  for (auto& v : B) v = (int8_t)(rand() % 255 - 127);
  int8_t *dA, *dB; int* dD;
  CK(hipMalloc(&dA, A.size())); CK(hipMalloc(&dB, B.size())); CK(hipMalloc(&dD, M * N * 4));
  CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipDeviceSynchronize());
  std::vector<int> D(M * N);
  CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      int s = 0;
      for (int k = 0; k < K; ++k) s += A[i * K + k] * B[j * K + k];
      if (s != D[i * N + j]) ++bad;
    }
  printf("layout %-12s mismatches %d / %d\n", name, bad, M * N);
  hipFree(dA); hipFree(dB); hipFree(dD);
  return bad;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s gcn %s CUs %d clock %d kHz\n", p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int bad = 0;
  bad += check("32x32x32", 32, 32, 32, k32x32x32);
  bad += check("16x16x64", 16, 16, 64, k16x16x64);
  bad += check("32x32x16", 32, 32, 16, k32x32x16);
  int *out; CK(hipMalloc(&out, 4096 * 256 * 4));
  const int iters = 20000, blocks = p.multiProcessorCount * 4;
  const char* names[3] = {"32x32x32_i8", "16x16x64_i8", "32x32x16_i8"};
  const double macs_per[3] = {32.0 * 32 * 32, 16.0 * 16 * 64, 32.0 * 32 * 16};
  for (int kind = 0; kind < 3; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      if (kind == 0) hipLaunchKernelGGL(rate<0>, dim3(blocks), dim3(256), 0, 0, iters, out, 3);
      if (kind == 1) hipLaunchKernelGGL(rate<1>, dim3(blocks), dim3(256), 0, 0, iters, out, 3);
      if (kind == 2) hipLaunchKernelGGL(rate<2>, dim3(blocks), dim3(256), 0, 0, iters, out, 3);
      hipEventRecord(b); CK(hipEventSynchronize(b));
      float ms; hipEventElapsedTime(&ms, a, b);
      double ops = 2.0 * macs_per[kind] * 4 * iters * blocks * 4;  // 4 waves/block, 4 mfma/iter
      if (rep) printf("rate %-12s %.1f ms  %.1f TOPS\n", names[kind], ms, ops / ms / 1e9);
    }
  }
  return bad ? 1 : 0;
}
