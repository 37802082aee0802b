// Timing probe (not product code): the 196-px stride-2 conv + fused
// downsample kernel (conv3x3s2i.hip) on the three ResNet-18 shapes, random
// int8 data, B = 256; argv: OW (28/14/7), dbg bits (2 = no LDS-DMA, 4 = no
// epilogues, 8 = no downsample epilogue, 16 / 32 = downsample / conv1 stores
// to a trash line), ds (1 default; 0 = conv1 alone).
// With -DDLQ_STAMPS it also prints per-wave s_memtime stamps (prologue,
// per-stage barrier wait / MFMA loop, epilogues) of three workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//          -I dlq_amd/csrc tools/probe/conv3x3s2i_probe.hip -o tools/probe/conv3x3s2i_probe
#define DLQ_ABLATION 1  // the kernel honours a.dbg (timing ablations)
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../dlq_amd/csrc/conv3x3s2i.hip"

using namespace dlq;
__global__ void fill_rand(int8_t* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (int8_t)((int)(x % 255u) - 127);
  }
}
int main(int argc, char** argv) {
  const int OW = argc > 1 ? atoi(argv[1]) : 7;
  const int dbg = argc > 2 ? atoi(argv[2]) : 0;
  const bool ds = argc > 3 ? atoi(argv[3]) != 0 : true;  // 0: conv1 alone (the engine's layer2.0 / layer3.0 since round 6)
  const int C = OW == 28 ? 64 : OW == 14 ? 128 : 256, OC = 2 * C, N = 256, W = 2 * OW;
  const size_t xin = (size_t)N * W * W * C, yout = (size_t)N * OW * OW * OC;
  const size_t wb = (size_t)OC * (C / 32) * 304, db = (size_t)OC * (C / 32) * 48;
  int8_t *x, *w, *wd, *y, *yd;
  float *al, *be;
  if (hipMalloc(&x, xin) || hipMalloc(&y, yout) || hipMalloc(&yd, yout) || hipMalloc(&w, wb) ||
      hipMalloc(&wd, db) || hipMalloc(&al, OC * 4) || hipMalloc(&be, OC * 4)) return 3;
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, x, xin, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, w, wb, 3u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, wd, db, 4u);
  std::vector<float> hal(OC, 1e-4f);
  if (hipMemcpy(al, hal.data(), OC * 4, hipMemcpyHostToDevice) || hipMemset(be, 0, OC * 4)) return 3;
  ConvArgs a{};
  a.x = x; a.w = w; a.alpha = al; a.beta = be; a.y = y;
  a.N = N; a.H = W; a.W = W; a.C = C; a.OH = OW; a.OW = OW; a.OC = OC; a.OCp = OC; a.K = 9 * C;
  a.kH = a.kW = 3; a.sH = a.sW = 2; a.pH = a.pW = 1; a.P = N * OW * OW; a.relu = 1; a.out_kind = 0; a.dbg = dbg;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 20; ++it) launch_conv3x3s2i(a, ds ? wd : nullptr, al, be, yd, 0);
  hipEventRecord(e0, 0);
  for (int it = 0; it < 20; ++it) launch_conv3x3s2i(a, ds ? wd : nullptr, al, be, yd, 0);
  hipEventRecord(e1, 0);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    printf("launch/sync failed\n");
    return 2;
  }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("OW=%d dbg=%d kernel %.1f us\n", OW, dbg, ms * 1e3 / 20);
#ifdef DLQ_STAMPS
  // per wave: prologue | per stage (barrier wait)/(MFMA loop) | epilogue, drain
  std::vector<unsigned long long> st(1024 * 8 * 64);
  if (hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps_j), st.size() * 8) != hipSuccess) return 2;
  const int NS = C / 32, nst = (OW == 28 ? 4 : OW == 14 ? 2 : 1) * NS;
  for (int blk : {0, 77, 200}) {
    for (int wv : {0, 4, 5}) {
      const unsigned long long* s = &st[(blk * 8 + wv) * 64];
      printf("blk %3d wave %d: pro %5llu (prep %llu issue %llu init %llu ->loop %llu vmwait %llu barrier %llu) |", blk, wv,
             s[1] - s[0], s[55] - s[0], s[56] - s[55], s[57] - s[56], s[58] - s[57], s[59] - s[58], s[1] - s[59]);
      for (int k = 0; k < nst; ++k)
        printf(" %llu/%llu", k ? s[1 + 2 * k] - s[2 * k] : 0ull, s[2 + 2 * k] - s[1 + 2 * k]);
      printf(" | tail %llu drain %llu total %llu\n", s[62] - s[2 * nst], s[63] - s[62], s[63] - s[0]);
    }
  }
#endif
  return 0;
}
