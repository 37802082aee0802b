// head.hip -- global average pool and dense (FC / MNIST MLP) layers.
//
// gap_kernel replaces gap_global / gap_global_ref (RK = CUDA/resnet18-kernel-
// lab/cpp/fp32: RK/kernels/gap_global.cu:2-33, RK/runtime/infer_e2e.cu:37-61)
// on int8 NHWC: exact int32 channel sums, then clamp(rne(float(sum) * k)).
// Each thread sums 16 channels over an eighth of the pixels with 16-byte
// loads (two in flight); the eight partial sums meet through three
// xor-shuffles.
//
// linear_kernel replaces fc_forward (RK/runtime/infer_e2e.cu:206-219:
// sgemm_tiled M=1000 N=1 K=512 + host bias) and the MNIST forward GEMMs
// (CUDA/MNIST_on_GPU/v4.cu:255-302, v5.cu:127-157): one wave per 32 output
// channels x 32 rows, v_mfma_i32_32x32x32_i8 over K with both fragments
// loaded straight from global memory (K is at most a few hundred bytes per
// row: no reuse worth staging), fused epilogue (int8 / fp32 / int32).  The
// weights are the generic packed image of a 1x1 conv (dlq_pack_conv_weights_s8).
#include "device_common.h"

namespace dlq {
namespace {

__global__ __launch_bounds__(256) void gap16_kernel(const int8_t* __restrict__ x, int N, int C, int HW, float k,
                                                    int8_t* __restrict__ y) {
  const int tpi = (C / 16) * 8;  // threads per image: 8 pixel groups per 16-channel group
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = (int)(t / tpi), r = (int)(t - (long)n * tpi);
  const int pg = r & 7, cg = r >> 3;
  int s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = 0;
  if (n < N) {
    const int8_t* src = x + (size_t)n * HW * C + cg * 16;
    int i = pg;
    for (; i + 8 < HW; i += 16) {  // two independent 16-byte loads in flight per step
      const v4i v0 = *(const v4i*)(src + (size_t)i * C);
      const v4i v1 = *(const v4i*)(src + (size_t)(i + 8) * C);
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          s[w * 4 + b] += (int)(signed char)(v0[w] >> (8 * b)) + (int)(signed char)(v1[w] >> (8 * b));
    }
    if (i < HW) {
      const v4i v = *(const v4i*)(src + (size_t)i * C);
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int b = 0; b < 4; ++b) s[w * 4 + b] += (int)(signed char)(v[w] >> (8 * b));
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    s[i] += __shfl_xor(s[i], 1);
    s[i] += __shfl_xor(s[i], 2);
    s[i] += __shfl_xor(s[i], 4);
  }
  if (n < N && pg == 0) {
    v4i o;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned u = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) u |= ((unsigned)sat_rne((float)s[w * 4 + b] * k) & 0xffu) << (8 * b);
      o[w] = (int)u;
    }
    *(v4i*)(y + (size_t)n * C + cg * 16) = o;
  }
}

// OUT: 0 int8 (optional ReLU), 1 fp32, 2 int32.
template <int OUT>
__global__ __launch_bounds__(64) void linear_kernel(const int8_t* __restrict__ x, int N, int K,
                                                    const int8_t* __restrict__ w, int OC, int OCp,
                                                    const float* __restrict__ alpha, const float* __restrict__ beta,
                                                    int relu, void* __restrict__ y) {
  const int lane = threadIdx.x, lr = lane & 31, lh = lane >> 5;
  const int ot = blockIdx.x, rt = blockIdx.y;
  const int oc = ot * 32 + lr, ol = oc & 63;
  const int row = min(rt * 32 + lr, N - 1);
  // generic packed image: [K/64][OCp/64][64 oc][4 x 16 B chunks at chunk ^ ((ol >> 2) & 3)]
  const int8_t* wp = w + ((size_t)(oc >> 6) * 64 + ol) * 64;
  const size_t wstride = (size_t)(OCp / 64) * 64 * 64;  // per 64-channel block
  const int sw = (ol >> 2) & 3;
  const int8_t* xp = x + (size_t)row * K + lh * 16;
  v16i acc = v16i{0};
  const int nk = K / 32;
  auto frag = [&](int kk, v4i& a, v4i& b) {
    const int lc = (2 * kk + lh) & 3;
    a = *(const v4i*)(wp + (size_t)(kk >> 1) * wstride + ((lc ^ sw) << 4));
    b = *(const v4i*)(xp + kk * 32);
  };
  int kk = 0;
  for (; kk + 4 <= nk; kk += 4) {  // four k-steps' loads in flight per MFMA group
    v4i a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) frag(kk + i, a[i], b[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[i], acc, 0, 0, 0);
  }
  for (; kk < nk; ++kk) {
    v4i a, b;
    frag(kk, a, b);
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
  }
  const int r = rt * 32 + lr;  // this lane's row (D column)
  if (r >= N) return;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int o0 = ot * 32 + 8 * g + 4 * lh;  // 4 consecutive output channels
    if constexpr (OUT == 2) {
      int* dst = (int*)y + (size_t)r * OC + o0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (o0 + e < OC) dst[e] = acc[4 * g + e];
    } else {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf((float)acc[4 * g + e], alpha[o0 + e], beta[o0 + e]);
      if constexpr (OUT == 1) {
        float* dst = (float*)y + (size_t)r * OC + o0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (o0 + e < OC) dst[e] = v[e];
      } else {
        if (o0 < OC) *(unsigned*)((int8_t*)y + (size_t)r * OC + o0) = quant4(v[0], v[1], v[2], v[3], relu ? 0.f : -127.f);
      }
    }
  }
}

// gap_fc_kernel: the network head (GAP + FC, RK/runtime/infer_e2e.cu:417-433)
// in ONE launch for C = K = 512, fp32 logits -- the same integers and the same
// float ops as gap16_kernel followed by linear_kernel<1>, so the logits are
// bit-identical.  Workgroup = GF images x 256 output channels (grid GF-image
// groups x 4: 256 workgroups at B = 256; the four workgroups of an image group
// have block ids 64 apart, i.e. the same XCD, so they share its L2 copy of the
// activations).  Phase 1: one wave per image, lane = (pixel parity, 16-channel
// group): a wave's load is 2 whole 512-byte pixel rows, every load of the
// image issued before the first sum, one v_permlane32_swap per sum joins the
// two parities; the int8 GAP codes go to LDS.  The first output tile's weight
// fragments are loaded before the activations, the second's behind them.
// Phase 2: each wave runs linear_kernel's MFMA loop for its two 32-channel
// tiles (two independent accumulator chains) with the B fragments read from
// LDS (lanes lr >= GF read a duplicate row; their D columns are not stored).
constexpr int GF = 4;        // images per workgroup (one per wave)
constexpr int GF_PR = 28;    // pixel loads per lane: HW <= 2 * GF_PR
constexpr int GF_OCW = 256;  // output channels per workgroup (4 waves x 2 tiles)

__global__ __launch_bounds__(256) void gap_fc_kernel(const int8_t* __restrict__ x, int N, int HW, float k,
                                                     const int8_t* __restrict__ w, int OC, int OCp,
                                                     const float* __restrict__ alpha, const float* __restrict__ beta,
                                                     float* __restrict__ y) {
  constexpr int C = 512, NK = C / 32;
  __shared__ __attribute__((aligned(16))) int8_t g[GF * C];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, lr = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.x * GF;
  const size_t wstride = (size_t)(OCp / 64) * 64 * 64;
  const int ot0 = (blockIdx.y * GF_OCW) / 32 + wv * 2;  // this wave's tiles ot0, ot0 + 1
  auto load_w = [&](int ot, v4i (&a)[NK]) {
    const int oc = min(ot * 32, OCp - 32) + lr, ol = oc & 63, sw = (ol >> 2) & 3;
    const int8_t* wp = w + ((size_t)(oc >> 6) * 64 + ol) * 64;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      a[kk] = *(const v4i*)(wp + (size_t)(kk >> 1) * wstride + ((((2 * kk + lh) & 3) ^ sw) << 4));
  };
  v4i a0[NK], a1[NK];
  load_w(ot0, a0);
  {
    const int cg = lane & 31, par = lane >> 5;
    const int n = min(n0 + wv, N - 1);  // a short last group re-reads a valid image
    const int8_t* src = x + (size_t)n * HW * C + cg * 16;
    v4i v[GF_PR];
#pragma unroll
    for (int j = 0; j < GF_PR; ++j) v[j] = *(const v4i*)(src + (size_t)min(par + 2 * j, HW - 1) * C);
    load_w(ot0 + 1, a1);
    int s[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = 0;
#pragma unroll
    for (int j = 0; j < GF_PR; ++j) {
      const bool ok = par + 2 * j < HW;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) s[q * 4 + b] += ok ? (int)(signed char)(v[j][q] >> (8 * b)) : 0;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      unsigned lo = (unsigned)s[e], hi = (unsigned)s[e];
      swap32(lo, hi);  // lanes 0-31: hi = the odd-pixel sum of the same channel group
      s[e] += (int)hi;
    }
    if (par == 0) {
      v4i o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        unsigned u = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) u |= ((unsigned)sat_rne((float)s[q * 4 + b] * k) & 0xffu) << (8 * b);
        o[q] = (int)u;
      }
      *(v4i*)(g + wv * C + cg * 16) = o;
    }
  }
  __syncthreads();

  const int8_t* gb = g + (lr & (GF - 1)) * C + lh * 16;
  v16i acc0 = v16i{0}, acc1 = v16i{0};
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    const v4i bf = *(const v4i*)(gb + kk * 32);
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[kk], bf, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[kk], bf, acc1, 0, 0, 0);
  }
  const int r = n0 + lr;
  if (lr >= GF || r >= N) return;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int ot = ot0 + tt;
    const v16i& acc = tt ? acc1 : acc0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o0 = ot * 32 + 8 * q + 4 * lh;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (o0 + e < OC) y[(size_t)r * OC + o0 + e] = __builtin_fmaf((float)acc[4 * q + e], alpha[o0 + e], beta[o0 + e]);
    }
  }
}

}  // namespace

// C = K = 512, HW <= 56 (the ResNet-18 head); hipErrorInvalidValue otherwise.
hipError_t launch_gap_fc(const int8_t* x, int N, int C, int HW, float k, const int8_t* w, int OC,
                         const float* alpha, const float* beta, float* y, hipStream_t s) {
  if (C != 512 || HW < 1 || HW > 2 * GF_PR || N < 1 || OC < 1) return hipErrorInvalidValue;
  const int OCp = packed_oc(OC);
  const dim3 grid((N + GF - 1) / GF, (OC + GF_OCW - 1) / GF_OCW);
  hipLaunchKernelGGL(gap_fc_kernel, grid, dim3(256), 0, s, x, N, HW, k, w, OC, OCp, alpha, beta, y);
  return hipGetLastError();
}

hipError_t launch_gap(const int8_t* x, int N, int C, int HW, float k, int8_t* y, hipStream_t s) {
  const long total = (long)N * (C / 16) * 8;
  hipLaunchKernelGGL(gap16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, N, C, HW, k, y);
  return hipGetLastError();
}

hipError_t launch_linear(const int8_t* x, int N, int K, const int8_t* w, int OC, const float* alpha,
                         const float* beta, int relu, int out_kind, void* y, hipStream_t s) {
  const int OCp = packed_oc(OC);
  const dim3 grid((OC + 31) / 32, (N + 31) / 32), block(64);
  if (out_kind == 1)
    hipLaunchKernelGGL(linear_kernel<1>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  else if (out_kind == 2)
    hipLaunchKernelGGL(linear_kernel<2>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  else
    hipLaunchKernelGGL(linear_kernel<0>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  return hipGetLastError();
}

}  // namespace dlq
