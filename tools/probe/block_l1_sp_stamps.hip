// Timing probe (not product code): section totals per wave of the
// software-pipelined int8 layer1 block kernel (block_l1_sp_kernel) at N=256 on
// random data.  Sections (s_memtime cycles): 0 phase setup, 1 jobs, 2 DMA
// issue + landing wait (conv1 waves), 3 barrier.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DDLQ_STAMPS \
//          -I dlq_amd/csrc tools/probe/block_l1_sp_stamps.hip -o tools/probe/block_l1_sp_stamps
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../dlq_amd/csrc/block_l1.hip"
namespace dlq {
std::atomic<int> g_knob_l1_grid{0};  // capi.cpp's knob (the probe links no library)
}

using namespace dlq;
int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 256;
  const size_t act = (size_t)N * 56 * 56 * 64;
  std::vector<int8_t> hx(act), hw(64 * 576);
  unsigned st = 12345;
  auto rnd = [&]() { st = st * 1103515245u + 12345u; return (int8_t)((st >> 16) & 0x7f); };
  for (auto& v : hx) v = rnd();
  for (auto& v : hw) v = (int8_t)(rnd() - 64);
  std::vector<float> al(64, 0.001f), be(64, 0.5f);
  int8_t *x, *y, *w;
  float *a, *bb;
  hipMalloc(&x, act); hipMalloc(&y, act); hipMalloc(&w, hw.size()); hipMalloc(&a, 256); hipMalloc(&bb, 256);
  hipMemcpy(x, hx.data(), act, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size(), hipMemcpyHostToDevice);
  hipMemcpy(a, al.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(bb, be.data(), 256, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it) launch_block_l1(x, N, w, a, bb, w, a, bb, 0.01f, y, 0);
  hipEventRecord(e0, 0);
  for (int it = 0; it < 20; ++it) launch_block_l1(x, N, w, a, bb, w, a, bb, 0.01f, y, 0);
  hipEventRecord(e1, 0);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) { printf("launch/sync failed\n"); return 2; }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("N=%d block_l1_sp %.1f us\n", N, ms * 1e3 / 20);
#ifdef DLQ_STAMPS
  std::vector<unsigned long long> s(256 * 8 * 128);
  hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_bstamps), s.size() * 8);
  for (int blk : {0, 77})
    for (int wv = 0; wv < 8; ++wv) {
      const unsigned long long* p = &s[(blk * 8 + wv) * 128];
      printf("blk %3d w%d: setup %7llu jobs %7llu dma %7llu barrier %7llu | total %llu\n", blk, wv, p[0], p[1], p[2],
             p[3], p[0] + p[1] + p[2] + p[3]);
    }
#endif
  return 0;
}
