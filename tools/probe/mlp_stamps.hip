// Timing probe (not product code): per-wave s_memtime stamps of the one-launch
// MLP (head.hip mlp_fused_kernel) at B = 1024, 784 x 128 x 10, random data;
// kernel time by hipEvents over 200 back-to-back launches at several B.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DDLQ_STAMPS \
//          -I dlq_amd/csrc tools/probe/mlp_stamps.hip -o tools/probe/mlp_stamps
#include <algorithm>
#include <cstdio>
#include <vector>
#include "../../dlq_amd/csrc/head.hip"
using namespace dlq;
int main() {
  const int in = 784, kp = 832, H = 128, OC = 10, NMAX = 1024;
  float *x, *a1, *b1, *a2, *b2, *y;
  int8_t *w1, *w2, *hq;
  std::vector<float> hx((size_t)NMAX * in);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u >> 7) % 2001) / 1000.f - 1.f;
  std::vector<int8_t> hw1((size_t)kp * 128), hw2((size_t)H * 64);
  for (size_t i = 0; i < hw1.size(); ++i) hw1[i] = (int8_t)((i * 7919) % 255 - 127);
  for (size_t i = 0; i < hw2.size(); ++i) hw2[i] = (int8_t)((i * 104729) % 255 - 127);
  std::vector<float> ha(128, 0.001f), hb(128, 0.5f);
  if (hipMalloc(&x, hx.size() * 4) || hipMalloc(&w1, hw1.size()) || hipMalloc(&w2, hw2.size()) ||
      hipMalloc(&a1, 512) || hipMalloc(&b1, 512) || hipMalloc(&a2, 512) || hipMalloc(&b2, 512) ||
      hipMalloc(&hq, (size_t)NMAX * H) || hipMalloc(&y, (size_t)NMAX * OC * 4))
    return 3;
  hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(w1, hw1.data(), hw1.size(), hipMemcpyHostToDevice);
  hipMemcpy(w2, hw2.data(), hw2.size(), hipMemcpyHostToDevice);
  for (float* p : {a1, b1, a2, b2}) hipMemcpy(p, (p == a1 || p == a2) ? ha.data() : hb.data(), 512, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mr : {16, 8, 4})
  for (int B : {16, 128, 1024}) {
    for (int i = 0; i < 20; ++i) launch_mlp_fused(x, B, in, kp, 1.f / 0.02f, w1, H, a1, b1, w2, OC, a2, b2, hq, y, 0, mr);
    hipEventRecord(e0, 0);
    for (int i = 0; i < 200; ++i) launch_mlp_fused(x, B, in, kp, 1.f / 0.02f, w1, H, a1, b1, w2, OC, a2, b2, hq, y, 0, mr);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("rows/wg %d B=%d: %.2f us per launch (back to back)\n", mr, B, ms * 1e3f / 200);
  }
  std::vector<unsigned long long> st(256 * 4 * 8);  // last run: rows/wg 4, B = 1024
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_mlp_stamps), st.size() * 8);
  const char* names[4] = {"start->w1/f2/ab issued", "->x quantised+barrier", "->fc1+epi+barrier", "->fc2 done"};
  for (int k = 0; k < 4; ++k) {
    std::vector<double> d;
    for (int w = 0; w < 256 * 4; ++w) d.push_back((double)(st[w * 8 + k + 1] - st[w * 8 + k]));
    std::sort(d.begin(), d.end());
    printf("%-26s median %.0f  p90 %.0f cycles (s_memtime)\n", names[k], d[d.size() / 2], d[d.size() * 9 / 10]);
  }
  std::vector<double> t0;
  for (int w = 0; w < 256 * 4; ++w) t0.push_back((double)st[w * 8]);
  std::sort(t0.begin(), t0.end());
  printf("wave start spread: %.0f cycles\n", t0.back() - t0.front());
  return 0;
}
