// Timing probe (not product code): the cost of the conv epilogue sequences
// of device_common.h in isolation -- 8 waves per workgroup (two per SIMD),
// one workgroup per CU, each wave requantising NF 32x32 int32 tiles (random
// accumulators in registers, alpha/beta from LDS) REPS times, the bytes
// folded into a checksum (no stores), s_memtime around the loop.
// argv: variant (0 relu: min + v_cvt_pk_u8_f32, 1 signed: med3 + magic add +
// perm, 2 relu via the magic path, 3 residual relu), tiles per wave.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
//          -I dlq_amd/csrc tools/probe/epi_probe.hip -o tools/probe/epi_probe
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_common.h"

using namespace dlq;

constexpr int REPS = 64;

template <int V, int NF>
__global__ __launch_bounds__(512, 1) void epi_kernel(const int* acc_in, const float* ab, unsigned* out,
                                                     unsigned long long* cyc) {
  __shared__ float lab[256];
  const int tid = threadIdx.x, lane = tid & 63, lh = lane >> 5;
  if (tid < 256) lab[tid] = ab[tid];
  __syncthreads();
  v16i acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[f][r] = acc_in[((blockIdx.x * 8 + (tid >> 6)) * NF + f) * 1024 + r * 64 + lane];
  float al[4][4], be[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      al[g][e] = lab[8 * g + 4 * lh + e];
      be[g][e] = lab[128 + 8 * g + 4 * lh + e];
    }
  unsigned sum = 0;
  const unsigned r4 = 0x81407f03u ^ (unsigned)lane;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < REPS; ++it) {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      unsigned q[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int a4[4] = {acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
        if constexpr (V == 0)
          q[g] = epi4_relu(a4, al[g], be[g]);
        else if constexpr (V == 1)
          q[g] = epi4(a4, al[g], be[g], -127.f);
        else if constexpr (V == 2)
          q[g] = epi4(a4, al[g], be[g], 0.f);
        else
          q[g] = epi4_res_relu(a4, al[g], be[g], r4 + g, 0.37f);
      }
      swap32(q[0], q[2]);
      swap32(q[1], q[3]);
      sum += q[0] ^ q[1] ^ q[2] ^ q[3];
      // keep the accumulators "fresh" each rep without extra VALU per value
      acc[f][it & 15] += 1;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + tid] = sum;
  if (lane == 0) cyc[blockIdx.x * 8 + (tid >> 6)] = t1 - t0;
}

template <int V, int NF>
double run(const int* acc, const float* ab, unsigned* out, unsigned long long* cyc, int nblk) {
  hipLaunchKernelGGL((epi_kernel<V, NF>), dim3(nblk), dim3(512), 0, 0, acc, ab, out, cyc);
  hipLaunchKernelGGL((epi_kernel<V, NF>), dim3(nblk), dim3(512), 0, 0, acc, ab, out, cyc);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  std::vector<unsigned long long> h(nblk * 8);
  if (hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  double s = 0;
  for (auto v : h) s += (double)v;
  return s / h.size() / REPS;  // cycles per wave per epilogue pass of NF tiles
}

int main(int argc, char** argv) {
  const int nblk = 256;
  int *acc;
  float* ab;
  unsigned* out;
  unsigned long long* cyc;
  std::vector<int> ha((size_t)nblk * 8 * 8 * 1024);
  for (size_t i = 0; i < ha.size(); ++i) ha[i] = (int)((i * 2654435761u) % 200000u) - 100000;
  std::vector<float> hab(256);
  for (int i = 0; i < 256; ++i) hab[i] = i < 128 ? 1e-3f * (1 + i % 7) : 0.25f * (i % 5);
  if (hipMalloc(&acc, ha.size() * 4) || hipMalloc(&ab, 1024) || hipMalloc(&out, nblk * 512 * 4) ||
      hipMalloc(&cyc, nblk * 8 * 8))
    return 3;
  if (hipMemcpy(acc, ha.data(), ha.size() * 4, hipMemcpyHostToDevice) ||
      hipMemcpy(ab, hab.data(), 1024, hipMemcpyHostToDevice))
    return 3;
  const char* names[4] = {"relu (min + cvt_pk_u8)", "signed (med3 + magic + perm)", "relu via med3/magic",
                          "residual relu"};
  for (int v = 0; v < 4; ++v) {
    double c4 = v == 0 ? run<0, 4>(acc, ab, out, cyc, nblk) : v == 1 ? run<1, 4>(acc, ab, out, cyc, nblk)
                : v == 2 ? run<2, 4>(acc, ab, out, cyc, nblk) : run<3, 4>(acc, ab, out, cyc, nblk);
    double c7 = v == 0 ? run<0, 7>(acc, ab, out, cyc, nblk) : v == 1 ? run<1, 7>(acc, ab, out, cyc, nblk)
                : v == 2 ? run<2, 7>(acc, ab, out, cyc, nblk) : run<3, 7>(acc, ab, out, cyc, nblk);
    printf("%-30s 4 tiles: %7.0f cyc/wave (%5.1f per tile)   7 tiles: %7.0f cyc/wave (%5.1f per tile)\n", names[v],
           c4, c4 / 4, c7, c7 / 7);
  }
  return 0;
}
