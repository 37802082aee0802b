// layerops.hip -- the per-layer C-ABI in the reference's own layout (NCHW,
// OIHW, row-major GEMM operands), for drop-in per-layer parity and for
// callers that drive layers one at a time like the reference's step drivers
// (RK = CUDA/resnet18-kernel-lab/cpp/fp32).
//
// These are the reference's extern "C" kernels and static host helpers
// (RK/include/utils.hpp:74-82, RK/runtime/infer_e2e.cu:64-219) restated for
// int8: the same argument order, NCHW semantics, the batch honoured, an
// explicit stream, int status returns (never exit).  The fused NHWC
// operators in capi.cpp / resnet18.cpp are the fast path; these wrappers
// convert layouts around them (dlq_conv2d_nchw_s8) or are simple HBM-bound
// kernels of their own.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dlq.h"
#include "device_common.h"

namespace dlq {
namespace {

int num_cus_layerops() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

inline unsigned grid1(size_t total, int per = 256) {
  size_t g = (total + per - 1) / per;
  if (g > 256 * 64) g = 256 * 64;
  return (unsigned)(g < 1 ? 1 : g);
}

__global__ void quantize_f32_s8_kernel(const float* __restrict__ x, size_t n, float inv_s, int8_t* __restrict__ q) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    q[i] = (int8_t)sat_rne(x[i] * inv_s);
}

// The HBM-streaming forms of the standalone quantise / dequant passes (x, q /
// acc, y 16-byte aligned; the scalar kernels above take the rest and the
// tails).  Grid = 8 workgroups of 256 per CU, each thread 4 independent
// 16-byte loads in flight per iteration (coalesced: consecutive lanes,
// consecutive 16-byte units), and the same per-element IEEE ops as the scalar
// kernels (sat_rne(x * inv_s); float(acc) * scale[c]): bit-identical.
constexpr int QV_UNROLL = 4;
__global__ __launch_bounds__(256) void quantize_f32_s8_v4_kernel(const float4* __restrict__ x, size_t n4, float inv_s,
                                                                 unsigned* __restrict__ q) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto q4 = [&](const float4 v) -> unsigned {
    return ((unsigned)sat_rne(v.x * inv_s) & 0xffu) | (((unsigned)sat_rne(v.y * inv_s) & 0xffu) << 8) |
           (((unsigned)sat_rne(v.z * inv_s) & 0xffu) << 16) | (((unsigned)sat_rne(v.w * inv_s) & 0xffu) << 24);
  };
  for (; i + (QV_UNROLL - 1) * stride < n4; i += QV_UNROLL * stride) {
    float4 v[QV_UNROLL];
#pragma unroll
    for (int u = 0; u < QV_UNROLL; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < QV_UNROLL; ++u) q[i + u * stride] = q4(v[u]);
  }
  for (; i < n4; i += stride) q[i] = q4(x[i]);
}

// HW % 4 == 0: a 16-byte group never crosses a channel row.  IDX: 32-bit
// index arithmetic when the element count allows it.
template <typename IDX>
__global__ __launch_bounds__(256) void dequant_s32_f32_v4_kernel(const int4* __restrict__ acc, IDX n4, IDX hw4, int C,
                                                                 const float* __restrict__ scale,
                                                                 float4* __restrict__ y) {
  const IDX stride = (IDX)gridDim.x * blockDim.x;
  IDX i = (IDX)blockIdx.x * blockDim.x + threadIdx.x;
  auto dq = [&](const int4 a, IDX j) -> float4 {
    const float s = scale[(int)((j / hw4) % (IDX)C)];
    return float4{(float)a.x * s, (float)a.y * s, (float)a.z * s, (float)a.w * s};
  };
  for (; i + (QV_UNROLL - 1) * stride < n4; i += QV_UNROLL * stride) {
    int4 a[QV_UNROLL];
#pragma unroll
    for (int u = 0; u < QV_UNROLL; ++u) a[u] = acc[i + u * stride];
#pragma unroll
    for (int u = 0; u < QV_UNROLL; ++u) y[i + u * stride] = dq(a[u], i + u * stride);
  }
  for (; i < n4; i += stride) y[i] = dq(acc[i], i);
}

inline unsigned grid_stream() { return 8u * (unsigned)num_cus_layerops(); }

template <typename T>
__global__ void nchw_to_nhwc_kernel(const T* __restrict__ x, int N, int C, int HW, int Cs, T* __restrict__ y) {
  const size_t total = (size_t)N * HW * Cs;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cs);
    const size_t np = i / Cs;
    const int p = (int)(np % HW), n = (int)(np / HW);
    y[i] = c < C ? x[((size_t)n * C + c) * HW + p] : (T)0;
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ x, int N, int C, int HW, T* __restrict__ y) {
  const size_t total = (size_t)N * C * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % HW);
    const size_t nc = i / HW;
    const int c = (int)(nc % C), n = (int)(nc / C);
    y[i] = x[((size_t)n * HW + p) * C + c];
  }
}

__global__ void bn_relu_requant_kernel(const int32_t* __restrict__ acc, int N, int C, int HW,
                                       const float* __restrict__ alpha, const float* __restrict__ beta, float lo,
                                       int8_t* __restrict__ y) {
  const size_t total = (size_t)N * C * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)((i / HW) % C);
    const float v = __builtin_fmaf((float)acc[i], alpha[c], beta[c]);
    y[i] = (int8_t)__builtin_rintf(__builtin_amdgcn_fmed3f(v, lo, 127.f));
  }
}

__global__ void add_relu_requant_kernel(const int8_t* __restrict__ a, const int8_t* __restrict__ r, size_t n,
                                        float a_s, float r_s, float lo, int8_t* __restrict__ y) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = __builtin_fmaf((float)r[i], r_s, (float)a[i] * a_s);
    y[i] = (int8_t)__builtin_rintf(__builtin_amdgcn_fmed3f(v, lo, 127.f));
  }
}

// maxpool2d_3x3_s2p1_nchw (RK/kernels/maxpool2d.cu:4-41) on int8 NCHW.
__global__ void maxpool_nchw_s8_kernel(const int8_t* __restrict__ x, int N, int C, int H, int W, int OH, int OW,
                                       int8_t* __restrict__ y) {
  const size_t total = (size_t)N * C * OH * OW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
    const size_t nc = i / ((size_t)OH * OW);
    const int8_t* p = x + nc * H * W;
    int m = -128;
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if ((unsigned)iw < (unsigned)W) m = max(m, (int)p[ih * W + iw]);
      }
    }
    y[i] = (int8_t)m;
  }
}

// gap_global (RK/kernels/gap_global.cu:2-33) on int8 NCHW: one wave per (n, c).
__global__ void gap_nchw_s8_kernel(const int8_t* __restrict__ x, int NC, int HW, float k, int8_t* __restrict__ y) {
  const int wave = (int)(((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (wave >= NC) return;
  int s = 0;
  for (int i = lane; i < HW; i += 64) s += x[(size_t)wave * HW + i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) y[wave] = (int8_t)sat_rne((float)s * k);
}

__global__ void dequant_s32_f32_kernel(const int32_t* __restrict__ acc, int N, int C, int HW,
                                       const float* __restrict__ scale, float* __restrict__ y) {
  const size_t total = (size_t)N * C * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
    y[i] = (float)acc[i] * scale[(i / HW) % C];
}

hipError_t launched() { return hipGetLastError(); }

int status(hipError_t e, const char* what) {
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
}

// Stored channel count of the NHWC conv for IC input channels: the RGB stem
// stores 4, the rest their own count.
int stored_c(int IC, int kH, int kW) { return (IC == 3 && kH == 7 && kW == 7) ? kStemC : IC; }

bool g_inited = false;

}  // namespace
}  // namespace dlq

using namespace dlq;

extern "C" {

int dlq_init(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hipDeviceProp_t p;
  if ((e = hipGetDeviceProperties(&p, device)) != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return fail(DLQ_ERR_STATE, std::string("dlq kernels are built for gfx950, device is ") + p.gcnArchName);
  g_inited = true;
  return DLQ_OK;
}

int dlq_finalize(void) {
  if (!g_inited) return DLQ_OK;
  g_inited = false;
  hipError_t e = hipDeviceSynchronize();
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "hipDeviceSynchronize");
}

int dlq_quantize_f32_s8(const float* x, size_t n, float inv_s, int8_t* q, void* stream) {
  if (n == 0) return DLQ_OK;
  if (!x || !q) return fail(DLQ_ERR_ARG, "quantize_f32_s8: null pointer");
  size_t n4 = 0;
  if (((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 3) == 0 && n >= 1024) {
    n4 = n / 4;
    hipLaunchKernelGGL(quantize_f32_s8_v4_kernel, dim3(grid_stream()), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)x, n4, inv_s, (unsigned*)q);
  }
  if (4 * n4 < n)
    hipLaunchKernelGGL(quantize_f32_s8_kernel, dim3(grid1(n - 4 * n4)), dim3(256), 0, (hipStream_t)stream, x + 4 * n4,
                       n - 4 * n4, inv_s, q + 4 * n4);
  return status(launched(), "quantize_f32_s8");
}

int dlq_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, void* stream) {
  if (M < 0 || N < 0 || K < 0) return fail(DLQ_ERR_ARG, "gemm_s8s8s32: negative size");
  if (M == 0 || N == 0) return DLQ_OK;
  if (!A || !B || !C) return fail(DLQ_ERR_ARG, "gemm_s8s8s32: null pointer");
  if ((long long)M * K >= (1LL << 31) || (long long)K * N >= (1LL << 31) || (long long)M * N >= (1LL << 31))
    return fail(DLQ_ERR_ARG, "gemm_s8s8s32: operand exceeds 2^31 elements");
  return status(launch_gemm_s8s8s32(A, B, C, M, N, K, (hipStream_t)stream), "gemm_s8s8s32");
}

int dlq_gemm_s8s8s32_nt(const int8_t* A, const int8_t* Bt, int32_t* C, int M, int N, int K, void* stream) {
  if (M < 0 || N < 0 || K < 0) return fail(DLQ_ERR_ARG, "gemm_s8s8s32_nt: negative size");
  if (M == 0 || N == 0) return DLQ_OK;
  if (!A || !Bt || !C) return fail(DLQ_ERR_ARG, "gemm_s8s8s32_nt: null pointer");
  if ((long long)M * K >= (1LL << 31) || (long long)K * N >= (1LL << 31) || (long long)M * N >= (1LL << 31))
    return fail(DLQ_ERR_ARG, "gemm_s8s8s32_nt: operand exceeds 2^31 elements");
  return status(launch_gemm_s8s8s32_nt(A, Bt, C, M, N, K, (hipStream_t)stream), "gemm_s8s8s32_nt");
}

size_t dlq_conv2d_nchw_workspace_bytes(int N, int IC, int H, int W, int OC, int kH, int kW, int sH, int sW, int pH,
                                       int pW) {
  const int Cs = stored_c(IC, kH, kW);
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  if (N < 0 || OH <= 0 || OW <= 0) return 0;
  const size_t wb = packed_bytes_for(Cs, OC, H, W, kH, kW, sH, sW, pH, pW);
  if (wb == 0) return 0;
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  // packed weights | NHWC input | NHWC output (int32-sized: any out_kind)
  return al(wb) + al((size_t)N * H * W * Cs) + al((size_t)N * OH * OW * OC * 4);
}

int dlq_conv2d_nchw_s8(const int8_t* x, int N, int IC, int H, int W, const int8_t* w_oihw, int OC, int kH, int kW,
                       int sH, int sW, int pH, int pW, const float* alpha, const float* beta, int relu, int out_kind,
                       void* y, void* workspace, size_t ws_bytes, void* stream, int* OH, int* OW) {
  if (!x || !w_oihw || !y || !OH || !OW) return fail(DLQ_ERR_ARG, "conv2d_nchw: null pointer");
  const int Cs = stored_c(IC, kH, kW);
  *OH = out_dim(H, kH, sH, pH);
  *OW = out_dim(W, kW, sW, pW);
  const size_t need = dlq_conv2d_nchw_workspace_bytes(N, IC, H, W, OC, kH, kW, sH, sW, pH, pW);
  if (need == 0) return fail(DLQ_ERR_ARG, "conv2d_nchw: unsupported shape");
  if (!workspace || ws_bytes < need) return fail(DLQ_ERR_ARG, "conv2d_nchw: workspace too small");
  if (N == 0) return DLQ_OK;
  hipStream_t s = (hipStream_t)stream;
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  const size_t wb = packed_bytes_for(Cs, OC, H, W, kH, kW, sH, sW, pH, pW);
  int8_t* wdev = (int8_t*)workspace;
  int8_t* xh = wdev + al(wb);
  void* yh = xh + al((size_t)N * H * W * Cs);
  // Weights per call, like the reference's per-call H2D (infer_e2e.cu:114-128).
  std::vector<int8_t> packed(wb);
  pack_conv_weights_for(Cs, OC, H, W, kH, kW, sH, sW, pH, pW, w_oihw, IC, packed.data());
  hipError_t e = hipMemcpyAsync(wdev, packed.data(), wb, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // `packed` dies at return
  if (e != hipSuccess) return hip_fail(e, "conv2d_nchw weight upload");
  const int HW = H * W;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel<int8_t>, dim3(grid1((size_t)N * HW * Cs)), dim3(256), 0, s, x, N, IC, HW,
                     Cs, xh);
  if ((e = launched()) != hipSuccess) return status(e, "conv2d_nchw transpose");
  dlq_conv_desc d{N, H, W, Cs, OC, kH, kW, sH, sW, pH, pW};
  int rc = dlq_conv2d_nhwc_s8(&d, xh, wdev, alpha, beta, nullptr, 0.f, relu, out_kind, yh, stream);
  if (rc) return rc;
  const int OHW = *OH * *OW;
  if (out_kind == DLQ_OUT_S8)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<int8_t>, dim3(grid1((size_t)N * OC * OHW)), dim3(256), 0, s,
                       (const int8_t*)yh, N, OC, OHW, (int8_t*)y);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<int32_t>, dim3(grid1((size_t)N * OC * OHW)), dim3(256), 0, s,
                       (const int32_t*)yh, N, OC, OHW, (int32_t*)y);
  return status(launched(), "conv2d_nchw transpose back");
}

int dlq_bn_relu_requant_s8(const int32_t* acc, int N, int C, int HW, const float* alpha, const float* beta, int relu,
                           int8_t* y, void* stream) {
  if (N < 0 || C <= 0 || HW <= 0) return fail(DLQ_ERR_ARG, "bn_relu_requant: bad shape");
  if (N == 0) return DLQ_OK;
  if (!acc || !alpha || !beta || !y) return fail(DLQ_ERR_ARG, "bn_relu_requant: null pointer");
  hipLaunchKernelGGL(bn_relu_requant_kernel, dim3(grid1((size_t)N * C * HW)), dim3(256), 0, (hipStream_t)stream,
                     acc, N, C, HW, alpha, beta, relu ? 0.f : -127.f, y);
  return status(launched(), "bn_relu_requant");
}

int dlq_add_relu_requant_s8(const int8_t* a, const int8_t* r, size_t n, float a_scale, float r_scale, int relu,
                            int8_t* y, void* stream) {
  if (n == 0) return DLQ_OK;
  if (!a || !r || !y) return fail(DLQ_ERR_ARG, "add_relu_requant: null pointer");
  hipLaunchKernelGGL(add_relu_requant_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, a, r, n, a_scale,
                     r_scale, relu ? 0.f : -127.f, y);
  return status(launched(), "add_relu_requant");
}

int dlq_maxpool2d_3x3_s2p1_nchw_s8(const int8_t* x, int N, int C, int H, int W, int8_t* y, void* stream) {
  if (N < 0 || C <= 0 || H <= 0 || W <= 0) return fail(DLQ_ERR_ARG, "maxpool_nchw: bad shape");
  if (N == 0) return DLQ_OK;
  if (!x || !y) return fail(DLQ_ERR_ARG, "maxpool_nchw: null pointer");
  const int OH = out_dim(H, 3, 2, 1), OW = out_dim(W, 3, 2, 1);
  hipLaunchKernelGGL(maxpool_nchw_s8_kernel, dim3(grid1((size_t)N * C * OH * OW)), dim3(256), 0,
                     (hipStream_t)stream, x, N, C, H, W, OH, OW, y);
  return status(launched(), "maxpool_nchw");
}

int dlq_gap_s8(const int8_t* x, int N, int C, int HW, float k, int8_t* y, void* stream) {
  if (N < 0 || C <= 0 || HW <= 0) return fail(DLQ_ERR_ARG, "gap: bad shape");
  if (N == 0) return DLQ_OK;
  if (!x || !y) return fail(DLQ_ERR_ARG, "gap: null pointer");
  const size_t waves = (size_t)N * C;
  hipLaunchKernelGGL(gap_nchw_s8_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x,
                     N * C, HW, k, y);
  return status(launched(), "gap");
}

int dlq_fc_s8(const int8_t* g, int N, int K, const int8_t* w_packed, int OC, const float* alpha, const float* bias,
              float* logits, void* stream) {
  return dlq_linear_s8(g, N, K, w_packed, OC, alpha, bias, 0, DLQ_OUT_F32, logits, stream);
}

int dlq_dequant_s32_f32(const int32_t* acc, int N, int C, int HW, const float* scale, float* y, void* stream) {
  if (N < 0 || C <= 0 || HW <= 0) return fail(DLQ_ERR_ARG, "dequant: bad shape");
  if (N == 0) return DLQ_OK;
  if (!acc || !scale || !y) return fail(DLQ_ERR_ARG, "dequant: null pointer");
  const size_t total = (size_t)N * C * HW;
  if (HW % 4 == 0 && ((uintptr_t)acc & 15) == 0 && ((uintptr_t)y & 15) == 0 && total >= 1024) {
    const size_t n4 = total / 4;
    if (n4 < 0x7fffffffu)
      hipLaunchKernelGGL(dequant_s32_f32_v4_kernel<unsigned>, dim3(grid_stream()), dim3(256), 0, (hipStream_t)stream,
                         (const int4*)acc, (unsigned)n4, (unsigned)(HW / 4), C, scale, (float4*)y);
    else
      hipLaunchKernelGGL(dequant_s32_f32_v4_kernel<size_t>, dim3(grid_stream()), dim3(256), 0, (hipStream_t)stream,
                         (const int4*)acc, n4, (size_t)(HW / 4), C, scale, (float4*)y);
  } else {
    hipLaunchKernelGGL(dequant_s32_f32_kernel, dim3(grid1(total)), dim3(256), 0, (hipStream_t)stream, acc, N, C, HW,
                       scale, y);
  }
  return status(launched(), "dequant");
}

}  // extern "C"
