// plan_capture.hip -- test infrastructure, not product code: the wide
// stride-1 conv (conv3x3i.hip) and the stride-2 conv + downsample
// (conv3x3s2i.hip) compiled with DLQ_PLAN_CAPTURE, so every LDS-DMA piece
// they would issue is recorded (device_common.h plan_capture) instead.  The
// kernels run their real launchers on device buffers of the real shapes;
// tests/test_gpu_dma_plan.py compares the recorded pieces (per workgroup and
// wave, in issue order: LDS address + 64 lane sources) with the plans
// tools/check/dma_plan.py derives, so the host checker cannot drift from the
// compiled kernels.
// Build (Makefile): compiled twice, -DPLANCAP_KIND=0 (wide) and 1 (stride-2),
// in parallel, and linked into tools/check/libplancap.so.
#define DLQ_PLAN_CAPTURE 1
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#if PLANCAP_KIND == 0
#include "../../dlq_amd/csrc/conv3x3i.hip"
#else
#include "../../dlq_amd/csrc/conv3x3s2i.hip"
#endif

using namespace dlq;

namespace {
template <typename T>
hipError_t dmalloc(T** p, size_t bytes) {
  return hipMalloc((void**)p, bytes ? bytes : 16);
}
}  // namespace

// kind 0: conv3x3i at W x W (C = OC from the ResNet-18 shape); kind 1:
// conv3x3s2i + fused downsample at input W x W (OW = W / 2).  Writes, per
// wave w of the launch (grid * 8 waves): cnt[w] pieces (at most max_rec),
// lds[w * max_rec + i], src[(w * max_rec + i) * 64 + lane]; bases = the
// device addresses of x, the conv weights, the downsample weights and the
// kernel's zero block.  Returns the number of waves, -1 on a HIP error, or -2
// if any piece went unrecorded (a wave past the buffers or past max_rec), -3
// if the launch has more waves than the caller's arrays (max_waves) hold.
#if PLANCAP_KIND == 0
#define PLANCAP_RUN plancap_run_wide
#else
#define PLANCAP_RUN plancap_run_s2i
#endif
extern "C" int PLANCAP_RUN(int kind, int W, int N, unsigned max_rec, unsigned* cnt, unsigned* lds,
                           unsigned long long* src, unsigned long long* bases, int max_waves) {
  if (kind != PLANCAP_KIND) return -1;
  const int C = kind == 0 ? (W == 28 ? 128 : W == 14 ? 256 : 512) : (W == 56 ? 64 : W == 28 ? 128 : 256);
  const int OW = kind == 0 ? W : W / 2, OC = kind == 0 ? C : 2 * C, P = N * OW * OW;
  const size_t xb = (size_t)N * W * W * C, yb = (size_t)P * OC;
  const size_t wb = kind == 0 ? (size_t)(C / 32) * (OC < 128 ? 128 : OC) * 304 : (size_t)(C / 32) * OC * 304;
  const size_t db = kind == 0 ? 0 : (size_t)(C / 32) * OC * 48;
  int8_t *x = nullptr, *w = nullptr, *wd = nullptr, *y = nullptr, *yd = nullptr;
  float* ab = nullptr;
  PlanPiece* buf = nullptr;
  unsigned* dcnt = nullptr;
  struct FreeAll {  // every exit path (HIP error, dropped pieces, success) frees the buffers
    void* const* p[8];
    ~FreeAll() {
      for (void* const* q : p)
        if (*q) (void)hipFree(*q);
    }
  } free_all{{(void* const*)&x, (void* const*)&w, (void* const*)&wd, (void* const*)&y, (void* const*)&yd,
               (void* const*)&ab, (void* const*)&buf, (void* const*)&dcnt}};
  const int items = kind == 0 ? (OC / (OW == 7 ? 64 : 128)) * ((P + 391) / 392) : (OC / 128) * ((P + 195) / 196);
  // the launchers' grid: min(items, CUs) (num_cus_i / num_cus_s2i)
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  const int grid = items < ncu ? items : ncu, nw = grid * 8;
  const unsigned nwu = (unsigned)nw, zero_u = 0;
  if (nw > max_waves) return -3;  // the caller's cnt / lds / src arrays hold max_waves waves
  if (dmalloc(&x, xb) || dmalloc(&w, wb) || dmalloc(&wd, db) || dmalloc(&y, yb) || dmalloc(&yd, yb) ||
      dmalloc(&ab, (size_t)4 * OC * 4) || dmalloc(&buf, (size_t)nw * max_rec * sizeof(PlanPiece)) ||
      dmalloc(&dcnt, (size_t)nw * 4))
    return -1;
  if (hipMemset(dcnt, 0, (size_t)nw * 4) || hipMemset(ab, 0, (size_t)4 * OC * 4)) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_cap_buf), &buf, sizeof(buf)) ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_cap_cnt), &dcnt, sizeof(dcnt)) ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_cap_max), &max_rec, sizeof(max_rec)) ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_cap_nw), &nwu, sizeof(nwu)) ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_cap_drop), &zero_u, sizeof(zero_u)))
    return -1;
  ConvArgs a{};
  a.x = x;
  a.w = w;
  a.alpha = ab;
  a.beta = ab + OC;
  a.y = y;
  a.N = N;
  a.H = a.W = W;
  a.C = C;
  a.OH = a.OW = OW;
  a.OC = a.OCp = OC;
  a.K = 9 * C;
  a.kH = a.kW = 3;
  a.sH = a.sW = kind == 0 ? 1 : 2;
  a.pH = a.pW = 1;
  a.P = P;
  a.relu = 1;
  a.out_kind = 0;
  void* zero = nullptr;
  hipError_t e;
#if PLANCAP_KIND == 0
  e = launch_conv3x3i(a, 0);
  if (e == hipSuccess) e = hipGetSymbolAddress(&zero, HIP_SYMBOL(g_zero_i));
#else
  e = launch_conv3x3s2i(a, wd, ab + 2 * OC, ab + 3 * OC, yd, 0);
  if (e == hipSuccess) e = hipGetSymbolAddress(&zero, HIP_SYMBOL(g_zero_s2i));
#endif
  if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned dropped = 0;
  if (hipMemcpyFromSymbol(&dropped, HIP_SYMBOL(g_cap_drop), sizeof(dropped)) != hipSuccess) return -1;
  if (dropped) return -2;  // a piece went unrecorded: the comparison would be incomplete
  std::vector<PlanPiece> h((size_t)nw * max_rec);
  if (hipMemcpy(h.data(), buf, h.size() * sizeof(PlanPiece), hipMemcpyDeviceToHost) ||
      hipMemcpy(cnt, dcnt, (size_t)nw * 4, hipMemcpyDeviceToHost))
    return -1;
  for (size_t i = 0; i < h.size(); ++i) {
    lds[i] = h[i].lds;
    for (int l = 0; l < 64; ++l) src[i * 64 + l] = h[i].src[l];
  }
  bases[0] = (uintptr_t)x;
  bases[1] = (uintptr_t)w;
  bases[2] = (uintptr_t)wd;
  bases[3] = (uintptr_t)zero;
  return nw;
}
