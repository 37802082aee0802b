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

}  // namespace

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
