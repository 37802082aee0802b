// Probe (not product code): the wide conv's steady-state stage loop in
// isolation (conv3x3i.hip: 8 waves per CU, SIMD pairs w / w+4 own 7 / 6
// tiles of one oc tile, 9 taps per stage, A fragment per tap + one B
// fragment per tile per tap from LDS, B re-read one tap ahead, one barrier
// per stage), on random int8 data already in LDS, no DMA and no epilogue.
// Variants isolate what keeps the loop from the MFMA pipe's rate:
//   0: as the kernel (LDS reads, barrier per stage)
//   1: no barrier
//   2: no LDS reads (fragments from registers), barrier per stage
//   3: no LDS reads, no barrier
//   4: LDS reads, barrier, B two taps ahead
//   5: LDS reads, barrier every 2 stages
// Output: TOPS and the in-kernel clock per variant.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/conv_loop_probe.hip -o tools/probe/conv_loop_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NF, int VAR>
__device__ __forceinline__ void body(const int8_t* lds, int nst, v16i (&acc)[7], const v4i* rf) {
  const int lane = threadIdx.x & 63;
  const int8_t* abase = lds + 40960 + (threadIdx.x >> 6) * 2048 + lane * 16;
  unsigned boff[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) boff[f] = (unsigned)(f * 3072 + lane * 16);
  for (int s = 0; s < nst; ++s) {
    const int8_t* sb = lds + (s & 1) * 512;
    if constexpr (VAR == 2 || VAR == 3) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(rf[tap & 3], rf[4 + ((f + tap) & 3)], acc[f], 0, 0, 0);
    } else if constexpr (VAR == 4) {
      v4i fa[2], fb[2][NF];
      fa[0] = *(const v4i*)(abase);
      fa[1] = *(const v4i*)(abase + 32);
#pragma unroll
      for (int f = 0; f < NF; ++f) fb[0][f] = *(const v4i*)(sb + boff[f]);
#pragma unroll
      for (int f = 0; f < NF; ++f) fb[1][f] = *(const v4i*)(sb + boff[f] + 16 * 64);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int bu = tap & 1;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu], fb[bu][f], acc[f], 0, 0, 0);
          if (f == NF - 1 && tap + 2 < 9) fa[bu] = *(const v4i*)(abase + (tap + 2) * 32);
          if (tap + 2 < 9) fb[bu][f] = *(const v4i*)(sb + boff[f] + (tap + 2) * 16 * 64 % 12288);
        }
      }
    } else {
      v4i fa[2], fb[NF];
      fa[0] = *(const v4i*)(abase);
#pragma unroll
      for (int f = 0; f < NF; ++f) fb[f] = *(const v4i*)(sb + boff[f]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int bu = tap & 1;
        if (tap + 1 < 9) fa[bu ^ 1] = *(const v4i*)(abase + (tap + 1) * 32);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu], fb[f], acc[f], 0, 0, 0);
          if (tap + 1 < 9) fb[f] = *(const v4i*)(sb + boff[f] + (tap + 1) * 16 * 64 % 12288);
        }
      }
    }
    if constexpr (VAR == 0 || VAR == 2 || VAR == 4) {
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    } else if constexpr (VAR == 5) {
      if (s & 1) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();
      }
    }
  }
}

template <int VAR>
__global__ __launch_bounds__(512, 1) void loop(const v4i* src, int nst, int* out, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) int8_t lds[65536];
  for (int i = threadIdx.x; i < 4096; i += 512) ((v4i*)lds)[i] = src[blockIdx.x * 64 + (i & 1023)];
  v4i rf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rf[i] = src[(blockIdx.x * 8 + i) * 64 + (threadIdx.x & 63)];
  __syncthreads();
  v16i acc[7] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x < 256)
    body<7, VAR>(lds, nst, acc, rf);
  else
    body<6, VAR>(lds, nst, acc, rf);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
#pragma unroll
  for (int f = 0; f < 7; ++f)
#pragma unroll
    for (int g = 0; g < 16; ++g) s += acc[f][g];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int VAR>
void run(const v4i* src, int* out, unsigned long long* clk) {
  const int G = 256, nst = 400;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0, 0);
    for (int l = 0; l < 20; ++l) hipLaunchKernelGGL(loop<VAR>, dim3(G), dim3(512), 0, 0, src, nst, out, clk);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(2 * G);
    hipMemcpy(c.data(), clk, 16 * G, hipMemcpyDeviceToHost);
    double ghz = 0, cyc = 0;
    for (int i = 0; i < G; ++i) {
      ghz += (double)c[2 * i] / (double)c[2 * i + 1] * 0.1;
      cyc += (double)c[2 * i];
    }
    ghz /= G;
    cyc /= G;
    const double mfma_per_simd = (double)nst * 9 * 13;  // both waves of a SIMD
    const double ops = 20.0 * G * 4 * mfma_per_simd * 65536.0;
    printf("var %d rep %d: %7.1f TOPS  clock %.3f GHz  %.1f stamp-cycles per stage (MFMA %d per SIMD)\n", VAR, rep,
           ops / (ms * 1e-3) / 1e12, ghz, cyc / nst, 117);
  }
}

int main() {
  std::vector<int> h(256 * 1024 * 4);
  unsigned x = 777;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (int)(x ^ (x >> 15));
  }
  v4i* src;
  int* out;
  unsigned long long* clk;
  if (hipMalloc(&src, h.size() * 4) || hipMalloc(&out, 256 * 512 * 4) || hipMalloc(&clk, 256 * 16) ||
      hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice))
    return 3;
  run<0>(src, out, clk);
  run<1>(src, out, clk);
  run<2>(src, out, clk);
  run<3>(src, out, clk);
  run<4>(src, out, clk);
  run<5>(src, out, clk);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
