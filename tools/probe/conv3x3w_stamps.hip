// Timing probe (not product code): per-wave s_memtime stamps of the wide
// stride-1 conv kernel on the layer4 shape, to locate where a stage's cycles go.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DDLQ_STAMPS \
//          -I dlq_amd/csrc tools/probe/conv3x3w_stamps.hip -o tools/probe/conv3x3w_stamps
#include <cstdio>
#include <cstdlib>
#include <vector>
namespace dlq {
int packed_oc(int OC) { return OC <= 64 ? 64 : (OC + 127) / 128 * 128; }
}
#include "../../dlq_amd/csrc/conv3x3w.hip"

using namespace dlq;
int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 7;
  const int dbg = argc > 2 ? atoi(argv[2]) : 0;
  const int C = W == 7 ? 512 : W == 14 ? 256 : 128, N = 256, P = N * W * W;
  int8_t *x, *w, *res, *y;
  float *al, *be;
  hipMalloc(&x, (size_t)P * C); hipMalloc(&res, (size_t)P * C); hipMalloc(&y, (size_t)P * C);
  hipMalloc(&w, conv3x3w_packed_bytes(C, C));
  hipMalloc(&al, C * 4); hipMalloc(&be, C * 4);
  hipMemset(x, 1, (size_t)P * C); hipMemset(res, 1, (size_t)P * C); hipMemset(w, 1, conv3x3w_packed_bytes(C, C));
  hipMemset(al, 0, C * 4); hipMemset(be, 0, C * 4);
  ConvArgs a{};
  a.x = x; a.w = w; a.alpha = al; a.beta = be; a.res = res; a.y = y; a.s_res = 0.01f;
  a.N = N; a.H = W; a.W = W; a.C = C; a.OH = W; a.OW = W; a.OC = C; a.OCp = C; a.K = 9 * C;
  a.kH = a.kW = 3; a.sH = a.sW = 1; a.pH = a.pW = 1; a.P = P; a.relu = 1; a.out_kind = 0; a.dbg = dbg;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int NI = (C / 128) * ((P + 255) / 256), grid = NI < 256 ? NI : 256;
  auto launch = [&]() {
#define XBCASE(v) \
  case v: \
    if (W == 7) hipLaunchKernelGGL((conv3x3w_kernel<7, 512, 0, true, v>), dim3(grid), dim3(WNW * 64), 0, 0, a); \
    else if (W == 14) hipLaunchKernelGGL((conv3x3w_kernel<14, 256, 0, true, v>), dim3(grid), dim3(WNW * 64), 0, 0, a); \
    else hipLaunchKernelGGL((conv3x3w_kernel<28, 128, 0, true, v>), dim3(grid), dim3(WNW * 64), 0, 0, a); \
    break;
    switch (dbg) { XBCASE(0) XBCASE(1) XBCASE(2) XBCASE(3) XBCASE(4) XBCASE(5) XBCASE(6) XBCASE(7) XBCASE(16) XBCASE(17) XBCASE(32) XBCASE(48) XBCASE(64) XBCASE(96) }
  };
  for (int it = 0; it < 3; ++it) launch();
  hipEventRecord(e0, 0);
  for (int it = 0; it < 10; ++it) launch();
  hipEventRecord(e1, 0);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    printf("launch/sync failed\n");
    return 2;
  }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("W=%d xb=%d kernel %.1f us\n", W, dbg, ms * 1e2);
#ifdef DLQ_STAMPS
  std::vector<unsigned long long> st(256 * 8 * 64);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  // block 0 wave 0 and a mid block: stamp deltas
  for (int blk : {0, 100}) {
    for (int wv : {0, 5}) {
      const unsigned long long* s = &st[(blk * 8 + wv) * 64];
      printf("blk %d wave %d: prologue %llu |", blk, wv, s[1] - s[0]);
      for (int k = 0; k < 16 && 4 + 3 * k < 63; ++k)
        printf(" [%llu %llu]", s[3 + 3 * k] - s[2 + 3 * k], s[4 + 3 * k] - s[3 + 3 * k]);
      printf(" end %llu total %llu\n", s[63] - s[4 + 3 * 15], s[63] - s[0]);
    }
  }
#endif
  return 0;
}
