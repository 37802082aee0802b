// Timing probe (not product code): section timers of the fused stem kernel at
// N=256 on random fp32 input.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DDLQ_STAMPS \
//          -I dlq_amd/csrc tools/probe/stem_stamps.hip -o tools/probe/stem_stamps
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../dlq_amd/csrc/stem.hip"

using namespace dlq;
int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 256;
  const size_t nx = (size_t)N * 3 * 224 * 224;
  std::vector<float> hx(nx);
  unsigned st = 1;
  for (auto& v : hx) { st = st * 1103515245u + 12345u; v = ((st >> 9) & 0xffff) / 32768.f - 1.f; }
  std::vector<int8_t> hw(64 * 256);
  for (auto& v : hw) { st = st * 1103515245u + 12345u; v = (int8_t)((st >> 16) & 0xff); }
  std::vector<float> al(64, 0.001f), be(64, 0.1f);
  float *x, *a, *b;
  int8_t *w, *y;
  hipMalloc(&x, nx * 4); hipMalloc(&w, hw.size()); hipMalloc(&a, 256); hipMalloc(&b, 256);
  hipMalloc(&y, (size_t)N * 56 * 56 * 64);
  hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size(), hipMemcpyHostToDevice);
  hipMemcpy(a, al.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(b, be.data(), 256, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it) launch_stem_fused(x, N, w, a, b, 20.f, y, 0);
  hipEventRecord(e0, 0);
  for (int it = 0; it < 20; ++it) launch_stem_fused(x, N, w, a, b, 20.f, y, 0);
  hipEventRecord(e1, 0);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) { printf("launch/sync failed\n"); return 2; }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("N=%d stem %.1f us\n", N, ms * 1e3 / 20);
#ifdef DLQ_STAMPS
  std::vector<unsigned long long> s(512 * 8 * 8);
  hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_sstamps), s.size() * 8);
  for (int blk : {0, 100})
    for (int wv = 0; wv < 8; ++wv) {
      const unsigned long long* p = &s[(blk * 8 + wv) * 8];
      printf("blk %3d w%d: barrier %7llu convert %7llu mfma-issue %6llu pool+epi %7llu store+load %7llu prologue %6llu\n", blk,
             wv, p[0], p[1], p[2], p[3], p[4], p[5]);
    }
#endif
  return 0;
}
