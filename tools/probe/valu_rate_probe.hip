// Timing probe (not product code): issue cost of the VALU instructions the
// conv epilogues use, 8 waves per CU (two per SIMD) each running 16
// independent copies of one instruction per iteration (inline asm, so the
// exact encoding is measured), s_memtime around the loop.  Prints cycles
// per instruction per wave and per SIMD (two waves).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/valu_rate_probe.hip -o tools/probe/valu_rate_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <utility>
#include <vector>

constexpr int ITERS = 256;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(512) void rate_kernel(float* out, unsigned long long* cyc, float seed) {
  float v[16];
  unsigned u[16];
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p2[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = seed + i + threadIdx.x;
    u[i] = __float_as_uint(v[i]) ^ (threadIdx.x * 7u);
    p2[i] = f2{v[i], v[i] + 1.f};
  }
  const float s = seed * 0.5f;
  const f2 s2 = f2{s, s + 0.25f};
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
#define OP10(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p2[i]) : "v"(s2));
#define OP11(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p2[i]) : "v"(s2));
#define OP12(i) asm volatile("v_mov_b32 %0, %1" : "=v"(v[i]) : "v"(v[(i + 5) & 15]));
#define OP13(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xa8" : "+v"(u[i]) : "v"(u[(i + 3) & 15]), "s"(0x7f7f7f7fu));
#define OP14(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
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
    if constexpr (OP == 10) { R16(OP10) }
    if constexpr (OP == 11) { R16(OP11) }
    if constexpr (OP == 12) { R16(OP12) }
    if constexpr (OP == 13) { R16(OP13) }
    if constexpr (OP == 14) { R16(OP14) }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += v[i] + (float)u[i] + p2[i][0] + p2[i][1];
  out[blockIdx.x * 512 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP>
double run(float* out, unsigned long long* cyc, int threads) {
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 1.5f);
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 1.5f);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  std::vector<unsigned long long> h(256 * 8, 0);
  if (hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  double s = 0;
  int n = 0;
  for (int b = 0; b < 256; ++b)
    for (int w = 0; w < threads / 64; ++w) s += (double)h[b * 8 + w], ++n;
  return s / n / (ITERS * 16.0);
}

template <int... OPS>
void run_all(float* out, unsigned long long* cyc, const char* const* names, std::integer_sequence<int, OPS...>) {
  for (int threads : {256, 512}) {
    printf("%d waves per SIMD\n", threads / 256);
    const double c[] = {run<OPS>(out, cyc, threads)...};
    for (int i = 0; i < (int)sizeof...(OPS); ++i)
      printf("  %-28s %6.2f cyc per instruction per wave (%5.2f per SIMD)\n", names[i], c[i], c[i] * 256 / threads);
  }
}

int main() {
  float* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 256 * 512 * 4) || hipMalloc(&cyc, 256 * 8 * 8)) return 3;
  const char* names[15] = {"v_cvt_f32_i32", "v_fma_f32", "v_min_f32 (literal)", "v_cvt_pk_u8_f32",
                           "v_permlane32_swap_b32", "v_med3_f32", "v_perm_b32", "v_cvt_f32_i32_sdwa (byte)",
                           "v_add_f32 (literal)", "v_min_f32 (vgpr)", "v_pk_fma_f32", "v_pk_add_f32", "v_mov_b32",
                           "v_bitop3_b32", "v_add_u32"};
  run_all(out, cyc, names, std::make_integer_sequence<int, 15>{});
  return 0;
}
