// Timing probe (not product code): per-wave s_memtime stamps of the 392-px
// wide stride-1 conv kernel (conv3x3i.hip), random int8 data; argv: W, dbg
// bits (2 no LDS-DMA, 4 no epilogue, 8 B fragments read for the first k-steps
// only, 256 stage 0's DMA issued twice: cold, then L2-hot), N, residual (0 = none; default on).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DDLQ_STAMPS \
//          -I dlq_amd/csrc tools/probe/conv3x3i_stamps.hip -o tools/probe/conv3x3i_stamps
#define DLQ_ABLATION 1  // the kernel honours a.dbg (timing ablations)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../dlq_amd/csrc/conv3x3i.hip"

using namespace dlq;
__global__ void fill_rand(int8_t* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (int8_t)((int)(x % 255u) - 127);
  }
}
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 7;
  const int dbg = argc > 2 ? atoi(argv[2]) : 0;
  const int C = W == 7 ? 512 : W == 14 ? 256 : 128, N = argc > 3 ? atoi(argv[3]) : 256, P = N * W * W;
  int8_t *x, *w, *res, *y;
  float *al, *be;
  const size_t wb = (size_t)C * (C / 32) * 304;
  if (hipMalloc(&x, (size_t)P * C) || hipMalloc(&res, (size_t)P * C) || hipMalloc(&y, (size_t)P * C) ||
      hipMalloc(&w, wb) || hipMalloc(&al, C * 4) || hipMalloc(&be, C * 4)) return 3;
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, x, (size_t)P * C, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, res, (size_t)P * C, 2u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, w, wb, 3u);
  std::vector<float> hal(C, 1e-4f);
  if (hipMemcpy(al, hal.data(), C * 4, hipMemcpyHostToDevice) || hipMemset(be, 0, C * 4)) return 3;
  ConvArgs a{};
  a.x = x; a.w = w; a.alpha = al; a.beta = be; a.res = (argc > 4 && atoi(argv[4]) == 0) ? nullptr : res; a.y = y; a.s_res = 0.01f;
  a.N = N; a.H = W; a.W = W; a.C = C; a.OH = W; a.OW = W; a.OC = C; a.OCp = C; a.K = 9 * C;
  a.kH = a.kW = 3; a.sH = a.sW = 1; a.pH = a.pW = 1; a.P = P; a.relu = 1; a.out_kind = 0; a.dbg = dbg;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 20; ++it) launch_conv3x3i(a, 0);
  hipEventRecord(e0, 0);
  for (int it = 0; it < 20; ++it) launch_conv3x3i(a, 0);
  hipEventRecord(e1, 0);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    printf("launch/sync failed\n");
    return 2;
  }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d dbg=%d kernel %.1f us\n", W, dbg, ms * 1e3 / 20);
#ifdef DLQ_STAMPS
  std::vector<unsigned long long> st(256 * 8 * 64);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps_i), st.size() * 8);
  const int NS = C / 32 / (W == 7 ? 2 : 1), nst = (W == 28 ? 2 : 1) * NS;
  for (int blk : {0, 77, 200}) {
    for (int wv : {0, 4, 5}) {
      const unsigned long long* s = &st[(blk * 8 + wv) * 64];
      printf("blk %3d wave %d: pro %5llu |", blk, wv, s[1] - s[0]);
      for (int k = 0; k < nst; ++k)
        printf(" %llu/%llu", k ? s[1 + 2 * k] - s[2 * k] : 0ull, s[2 + 2 * k] - s[1 + 2 * k]);
      printf(" | epi %llu drain %llu total %llu", s[62] - s[2 * nst], s[63] - s[62], s[63] - s[0]);
      if (dbg & 256) printf(" | stage-0 DMA cold %llu, again (L2-hot) %llu", s[60] - s[0], s[61] - s[60]);
      printf("\n");
    }
  }
#endif
  return 0;
}
