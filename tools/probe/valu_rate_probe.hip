// Timing probe (not product code): issue cost of the VALU instructions the
// conv epilogues use, 8 waves per CU (two per SIMD) each running 16
// independent copies of one instruction per iteration (inline asm, so the
// exact encoding is measured), s_memtime around the loop.  Prints cycles
// per instruction per wave and per SIMD (two waves).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/valu_rate_probe.hip -o tools/probe/valu_rate_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int ITERS = 256;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(512, 1) void rate_kernel(float* out, unsigned long long* cyc, float seed) {
  float v[16];
  unsigned u[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = seed + i + threadIdx.x;
    u[i] = __float_as_uint(v[i]) ^ (threadIdx.x * 7u);
  }
  const float s = seed * 0.5f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#define OP0(i) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(v[i]));
#define OP1(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(s));
#define OP2(i) asm volatile("v_min_f32 %0, 0x42fe0000, %0" : "+v"(v[i]));
#define OP3(i) asm volatile("v_cvt_pk_u8_f32 %0, %1, 1, %0" : "+v"(u[i]) : "v"(v[i]));
#define OP4(i) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(u[i]), "+v"(u[(i + 1) & 15]));
#define OP5(i) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "s"(s), "v"(s));
#define OP6(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 3) & 15]), "s"(0x0c0c0400u));
#define OP7(i) asm volatile("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(v[i]) : "v"(u[i]));
#define OP8(i) asm volatile("v_add_f32 %0, 0x4b400000, %0" : "+v"(v[i]));
#define OP9(i) asm volatile("v_min_f32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
    if constexpr (OP == 0) { R16(OP0) }
    if constexpr (OP == 1) { R16(OP1) }
    if constexpr (OP == 2) { R16(OP2) }
    if constexpr (OP == 3) { R16(OP3) }
    if constexpr (OP == 4) { R16(OP4) }
    if constexpr (OP == 5) { R16(OP5) }
    if constexpr (OP == 6) { R16(OP6) }
    if constexpr (OP == 7) { R16(OP7) }
    if constexpr (OP == 8) { R16(OP8) }
    if constexpr (OP == 9) { R16(OP9) }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += v[i] + (float)u[i];
  out[blockIdx.x * 512 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP>
double run(float* out, unsigned long long* cyc) {
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(256), dim3(512), 0, 0, out, cyc, 1.5f);
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(256), dim3(512), 0, 0, out, cyc, 1.5f);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  std::vector<unsigned long long> h(256 * 8);
  if (hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  double s = 0;
  for (auto x : h) s += (double)x;
  return s / h.size() / (ITERS * 16.0);
}

int main() {
  float* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 256 * 512 * 4) || hipMalloc(&cyc, 256 * 8 * 8)) return 3;
  const char* names[10] = {"v_cvt_f32_i32", "v_fma_f32", "v_min_f32 (literal)", "v_cvt_pk_u8_f32",
                           "v_permlane32_swap_b32", "v_med3_f32", "v_perm_b32", "v_cvt_f32_i32_sdwa (byte)",
                           "v_add_f32 (literal)", "v_min_f32 (vgpr)"};
  double c[10] = {run<0>(out, cyc), run<1>(out, cyc), run<2>(out, cyc), run<3>(out, cyc), run<4>(out, cyc),
                  run<5>(out, cyc), run<6>(out, cyc), run<7>(out, cyc), run<8>(out, cyc), run<9>(out, cyc)};
  for (int i = 0; i < 10; ++i)
    printf("%-28s %6.2f cyc per instruction per wave (two waves per SIMD: %5.2f per SIMD)\n", names[i], c[i],
           c[i] / 2);
  return 0;
}
