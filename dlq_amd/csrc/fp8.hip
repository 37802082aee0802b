// fp8.hip -- the e4m3 (OCP fp8) variant of the inference path: BASELINE
// configs[4] "per-channel weights + fp8 activations on CDNA4 fp8 MFMA",
// SURVEY.md §8(f) row 4.  The reference has no fp8 code; the scheme is the
// build's own and oracle/oracle.c ora_*_f8 define it.
//
// Scheme: activations are e4m3 codes at a per-tensor scale (amax/448),
// weights e4m3 per output channel (max|w|/448); MFMA products are exact and
// accumulate in fp32 (v_mfma_f32_32x32x64_f8f6f4, kernels.hip conv_s8_kernel
// <..., F8>); the epilogue is the int8 one with the rounding replaced by
// clamp(y, lo, 448) -> e4m3 round-to-nearest-even (enc4_f8).
//
// This file: the HBM-bound passes around the convs (quantise, GAP) and the
// FC head, plus the fp8 C-ABI.  GAP sums exact integer units (every e4m3
// value is a multiple of 2^-9), the FC accumulates exact products in fp64,
// so both are bit-identical to the oracle; only the convs' fp32 MFMA
// accumulation is inexact (tests/test_gpu_f8.py states the tolerance).
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "../../include/dlq.h"
#include "device_common.h"

namespace dlq {
namespace {

// e4m3 byte -> value * 512 (an exact integer); v_cvt_f32_fp8 then a
// power-of-two scale.
__device__ __forceinline__ int f8_units(int word, int sel) {
  float v;
  switch (sel) {
    case 0: v = __builtin_amdgcn_cvt_f32_fp8(word, 0); break;
    case 1: v = __builtin_amdgcn_cvt_f32_fp8(word, 1); break;
    case 2: v = __builtin_amdgcn_cvt_f32_fp8(word, 2); break;
    default: v = __builtin_amdgcn_cvt_f32_fp8(word, 3); break;
  }
  return (int)(v * 512.f);
}

// Flat fp32 -> e4m3: q = requant(x * inv_s, -448); 4 values per thread.
__global__ __launch_bounds__(256) void quantize_f8_kernel(const float* __restrict__ x, size_t n, float inv_s,
                                                          uint8_t* __restrict__ y) {
  const size_t n4 = n / 4;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += (size_t)gridDim.x * blockDim.x) {
    const float4 v = *(const float4*)(x + 4 * t);
    *(unsigned*)(y + 4 * t) = enc4_f8(v.x * inv_s, v.y * inv_s, v.z * inv_s, v.w * inv_s, -448.f);
  }
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n - 4 * n4) {
    const size_t i = 4 * n4 + t;
    y[i] = (uint8_t)enc4_f8(x[i] * inv_s, 0.f, 0.f, 0.f, -448.f);
  }
}

// fp32 NCHW RGB -> e4m3 NHWC4 (channel 3 = +0): one thread = 4 pixels.
__global__ __launch_bounds__(256) void quantize_rgb_nhwc4_f8_kernel(const float* __restrict__ x, int N, int H, int W,
                                                                    float inv_s, uint8_t* __restrict__ y) {
  const int W4 = W >> 2;
  const long total = (long)N * H * W4;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int w4 = (int)(t % W4);
    const long nh = t / W4;
    const int h = (int)(nh % H), n = (int)(nh / H);
    const size_t plane = (size_t)H * W;
    const float* src = x + (size_t)n * 3 * plane + (size_t)h * W + 4 * w4;
    const float4 r = *(const float4*)(src);
    const float4 g = *(const float4*)(src + plane);
    const float4 b = *(const float4*)(src + 2 * plane);
    v4i out;
    out[0] = (int)enc4_f8(r.x * inv_s, g.x * inv_s, b.x * inv_s, 0.f, -448.f);
    out[1] = (int)enc4_f8(r.y * inv_s, g.y * inv_s, b.y * inv_s, 0.f, -448.f);
    out[2] = (int)enc4_f8(r.z * inv_s, g.z * inv_s, b.z * inv_s, 0.f, -448.f);
    out[3] = (int)enc4_f8(r.w * inv_s, g.w * inv_s, b.w * inv_s, 0.f, -448.f);
    *(v4i*)(y + ((size_t)(n * H + h) * W + 4 * w4) * 4) = out;
  }
}

// Generic fp32 NCHW -> e4m3 NHWC (Cout >= C, padding channels +0).
__global__ __launch_bounds__(256) void quantize_nchw_nhwc_f8_kernel(const float* __restrict__ x, int N, int C, int H,
                                                                    int W, int Cout, float inv_s,
                                                                    uint8_t* __restrict__ y) {
  const long total = (long)N * H * W * Cout;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % Cout);
    const long pix = t / Cout;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H), n = (int)(nh / H);
    const float v = c < C ? x[(((size_t)n * C + c) * H + h) * W + w] * inv_s : 0.f;
    y[t] = (uint8_t)enc4_f8(v, 0.f, 0.f, 0.f, -448.f);
  }
}

// GAP on e4m3 NHWC: one thread = 4 channels of one image; exact integer unit
// sums, y = requant(float(S) * k) (k already includes the 2^-9 unit scale).
__global__ __launch_bounds__(256) void gap_f8_kernel(const uint8_t* __restrict__ x, int N, int C, int HW, float k,
                                                     uint8_t* __restrict__ y) {
  const int c4 = C >> 2;
  const long total = (long)N * c4;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % c4), n = (int)(t / c4);
    const uint8_t* src = x + (size_t)n * HW * C + 4 * cg;
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < HW; ++i) {
      const int d = *(const int*)(src + (size_t)i * C);
      s0 += f8_units(d, 0);
      s1 += f8_units(d, 1);
      s2 += f8_units(d, 2);
      s3 += f8_units(d, 3);
    }
    *(unsigned*)(y + (size_t)n * C + 4 * cg) =
        enc4_f8((float)s0 * k, (float)s1 * k, (float)s2 * k, (float)s3 * k, -448.f);
  }
}

// FC on e4m3: logits[n][o] = fmaf(float(acc), alpha[o], beta[o]) with the
// exact acc = sum_k x[n][k] * w[o][k] accumulated in fp64 (every partial sum
// is a multiple of 2^-18 below 2^35: exact).  Block = 256 outputs o x 4
// images; the 4 image rows are decoded once into LDS.
constexpr int kFcImgs = 4;
__global__ __launch_bounds__(256) void linear_f8_kernel(const uint8_t* __restrict__ x, int N, int K,
                                                        const uint8_t* __restrict__ w, int O,
                                                        const float* __restrict__ alpha,
                                                        const float* __restrict__ beta, float* __restrict__ y) {
  extern __shared__ float xs[];  // [kFcImgs][K]
  const int n0 = blockIdx.y * kFcImgs, o = blockIdx.x * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < kFcImgs * K; i += 256) {
    const int r = i / K, c = i - r * K;
    xs[i] = n0 + r < N ? __builtin_amdgcn_cvt_f32_fp8((int)x[(size_t)(n0 + r) * K + c], 0) : 0.f;
  }
  __syncthreads();
  if (o >= O) return;
  double acc[kFcImgs] = {0.0, 0.0, 0.0, 0.0};
  const uint8_t* wr = w + (size_t)o * K;
  for (int k = 0; k < K; k += 4) {
    const int d = *(const int*)(wr + k);
    const double wv[4] = {(double)__builtin_amdgcn_cvt_f32_fp8(d, 0), (double)__builtin_amdgcn_cvt_f32_fp8(d, 1),
                          (double)__builtin_amdgcn_cvt_f32_fp8(d, 2), (double)__builtin_amdgcn_cvt_f32_fp8(d, 3)};
#pragma unroll
    for (int r = 0; r < kFcImgs; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[r] = __builtin_fma(wv[j], (double)xs[r * K + k + j], acc[r]);
  }
#pragma unroll
  for (int r = 0; r < kFcImgs; ++r)
    if (n0 + r < N) y[(size_t)(n0 + r) * O + o] = __builtin_fmaf((float)acc[r], alpha[o], beta[o]);
}

// GAP for C % 16 == 0 (the network's shape): head.hip's gap16 structure --
// one thread = 16 channels x an eighth of the pixels, two 16-byte loads in
// flight, three xor-shuffles -- on exact integer unit sums (the same sums as
// gap_f8_kernel, so the same result).
__device__ __forceinline__ void add_units16(int* s, const v4i v) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    s[4 * w + 0] += f8_units(v[w], 0);
    s[4 * w + 1] += f8_units(v[w], 1);
    s[4 * w + 2] += f8_units(v[w], 2);
    s[4 * w + 3] += f8_units(v[w], 3);
  }
}

__global__ __launch_bounds__(256) void gap16_f8_kernel(const uint8_t* __restrict__ x, int N, int C, int HW, float k,
                                                       uint8_t* __restrict__ y) {
  const int tpi = (C / 16) * 8;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = (int)(t / tpi), r = (int)(t - (long)n * tpi);
  const int pg = r & 7, cg = r >> 3;
  int s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = 0;
  if (n < N) {
    const uint8_t* src = x + (size_t)n * HW * C + cg * 16;
    int i = pg;
    for (; i + 8 < HW; i += 16) {
      const v4i v0 = *(const v4i*)(src + (size_t)i * C);
      const v4i v1 = *(const v4i*)(src + (size_t)(i + 8) * C);
      add_units16(s, v0);
      add_units16(s, v1);
    }
    if (i < HW) add_units16(s, *(const v4i*)(src + (size_t)i * C));
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
    for (int w = 0; w < 4; ++w)
      o[w] = (int)enc4_f8((float)s[4 * w] * k, (float)s[4 * w + 1] * k, (float)s[4 * w + 2] * k,
                          (float)s[4 * w + 3] * k, -448.f);
    *(v4i*)(y + (size_t)n * C + cg * 16) = o;
  }
}

// FC for K % 64 == 0 on v_mfma_f64_16x16x4f64: the e4m3 codes are decoded to
// fp64 (exact) and every partial sum is a multiple of 2^-18 below 2^35, so
// the f64 MFMA's sums are exact in any order -- the same acc as
// linear_f8_kernel.  One wave = 16 rows n x 16 outputs o; each lane streams
// 16-byte pieces of one x row and one w row, and MFMA s of a 64-deep chunk
// takes byte s of every lane's 16-byte piece (the same k for A and B).
// Block = 4 waves = 16 rows x 64 outputs.
__global__ __launch_bounds__(256) void linear_f8_mfma_kernel(const uint8_t* __restrict__ x, int N, int K,
                                                             const uint8_t* __restrict__ w, int O,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ beta, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * 16, o0 = blockIdx.x * 64 + wave * 16;
  const int n = min(n0 + li, N - 1), o = min(o0 + li, O - 1);
  const uint8_t* xr = x + (size_t)n * K + g * 16;
  const uint8_t* wr = w + (size_t)o * K + g * 16;
  typedef double v4d __attribute__((ext_vector_type(4)));
  v4d acc = {0.0, 0.0, 0.0, 0.0};
  auto dec = [](int word, int sel) -> double {
    float v;
    switch (sel) {
      case 0: v = __builtin_amdgcn_cvt_f32_fp8(word, 0); break;
      case 1: v = __builtin_amdgcn_cvt_f32_fp8(word, 1); break;
      case 2: v = __builtin_amdgcn_cvt_f32_fp8(word, 2); break;
      default: v = __builtin_amdgcn_cvt_f32_fp8(word, 3); break;
    }
    return (double)v;
  };
  v4i xa = *(const v4i*)xr, wb = *(const v4i*)wr;
  for (int k0 = 0; k0 < K; k0 += 64) {
    const v4i xc = xa, wc = wb;
    if (k0 + 64 < K) {  // next chunk's pieces in flight during this chunk's MFMAs
      xa = *(const v4i*)(xr + k0 + 64);
      wb = *(const v4i*)(wr + k0 + 64);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(dec(xc[s >> 2], s & 3), dec(wc[s >> 2], s & 3), acc, 0, 0, 0);
  }
  // D[i][j] (f64 layout, cdna_hip_programming.md): row i = n (g + 4 * e), column j = o (li)
  const int oc = o0 + li;
  if (oc >= O) return;
  const float al = alpha[oc], be = beta[oc];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int nr = n0 + g + 4 * e;
    if (nr < N) y[(size_t)nr * O + oc] = __builtin_fmaf((float)acc[e], al, be);
  }
}

int grid_for(long total) {
  long g = (total + 255) / 256;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

int launch_result(const char* what) {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// Host e4m3 encoder (weight quantisation), op for op oracle.c f8_encode.
uint8_t f8_encode_host(float y) {
  const uint8_t sgn = std::signbit(y) ? 0x80 : 0;
  const float a = std::fabs(y);
  uint8_t code;
  if (a < 0x1p-6f) {
    code = (uint8_t)(int)std::nearbyint(a * 512.f);
  } else {
    int e;
    std::frexp(a, &e);
    const int E = e - 1;
    int r = (int)std::nearbyint(std::ldexp(a, 3 - E));
    int eb = E + 7;
    if (r == 16) {
      r = 8;
      ++eb;
    }
    code = (uint8_t)((eb << 3) | (r - 8));
  }
  return code | sgn;
}

uint8_t f8_requant_host(float y, float lo) {
  y = y < lo ? lo : y;
  y = y > 448.f ? 448.f : y;
  return f8_encode_host(y + 0.0f);
}

// The wide kernels' shapes take their image; every other fp8 conv the generic one.
bool f8_wide(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  return conv3x3w_shape(C, OC, H, W, kH, kW, sH, sW, pH, pW) || conv3x3s2_shape(C, OC, H, W, kH, kW, sH, sW, pH, pW);
}

namespace {
hipError_t launch_wide_f8(const ConvArgs& a, hipStream_t s) {
  return a.sH == 2 ? launch_conv3x3s2i_f8(a, nullptr, nullptr, nullptr, nullptr, s) : launch_conv3x3i_f8(a, s);
}
}  // namespace

size_t packed_bytes_f8(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  if (f8_wide(C, OC, H, W, kH, kW, sH, sW, pH, pW)) return conv3x3w_packed_bytes(OC, C);
  return packed_bytes(OC, C, kH, kW);
}

void pack_conv_weights_f8(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW,
                          const uint8_t* q, int IC, uint8_t* packed) {
  if (f8_wide(C, OC, H, W, kH, kW, sH, sW, pH, pW))
    conv3x3w_pack((const int8_t*)q, OC, IC, C, (int8_t*)packed);
  else
    pack_conv_weights((const int8_t*)q, OC, IC, kH, kW, C, (int8_t*)packed);
}

void quantize_weights_f8(const float* w, int OC, int K, uint8_t* q, float* scale) {
  for (int o = 0; o < OC; ++o) {
    float mx = 0.f;
    for (int k = 0; k < K; ++k) {
      const float a = std::fabs(w[(size_t)o * K + k]);
      mx = a > mx ? a : mx;
    }
    const float s = mx > 0.f ? mx / 448.f : 1.f;
    scale[o] = s;
    for (int k = 0; k < K; ++k) q[(size_t)o * K + k] = f8_requant_host(w[(size_t)o * K + k] / s, -448.f);
  }
}

}  // namespace dlq

using namespace dlq;

extern "C" {

int dlq_quantize_weights_f8(const float* w, int OC, int K, uint8_t* q, float* scale) {
  if (!w || !q || !scale || OC <= 0 || K <= 0) return fail(DLQ_ERR_ARG, "quantize_weights_f8: bad args");
  quantize_weights_f8(w, OC, K, q, scale);
  return DLQ_OK;
}

int dlq_quantize_f32_f8(const float* x, size_t n, float inv_s, uint8_t* q, void* stream) {
  if (n == 0) return DLQ_OK;
  if (!x || !q) return fail(DLQ_ERR_ARG, "quantize_f32_f8: null pointer");
  if (((uintptr_t)x & 15) || ((uintptr_t)q & 3)) return fail(DLQ_ERR_ARG, "quantize_f32_f8: misaligned buffer");
  hipLaunchKernelGGL(quantize_f8_kernel, dim3(grid_for((long)(n / 4 + 1))), dim3(256), 0, (hipStream_t)stream, x, n,
                     inv_s, q);
  return launch_result("quantize_f32_f8");
}

int dlq_quantize_nchw_to_nhwc_f8(const float* x, int N, int C, int H, int W, int Cout, float inv_s, uint8_t* y,
                                 void* stream) {
  if (!x || !y || N < 0 || C <= 0 || Cout < C || H <= 0 || W <= 0)
    return fail(DLQ_ERR_ARG, "quantize_nchw_to_nhwc_f8: bad args");
  if (N == 0) return DLQ_OK;
  if (C == 3 && Cout == 4 && W % 4 == 0) {
    hipLaunchKernelGGL(quantize_rgb_nhwc4_f8_kernel, dim3(grid_for((long)N * H * (W / 4))), dim3(256), 0,
                       (hipStream_t)stream, x, N, H, W, inv_s, y);
  } else {
    hipLaunchKernelGGL(quantize_nchw_nhwc_f8_kernel, dim3(grid_for((long)N * H * W * Cout)), dim3(256), 0,
                       (hipStream_t)stream, x, N, C, H, W, Cout, inv_s, y);
  }
  return launch_result("quantize_nchw_to_nhwc_f8");
}

#define F8_GEOM(d) (d)->C, (d)->OC, (d)->H, (d)->W, (d)->kH, (d)->kW, (d)->sH, (d)->sW, (d)->pH, (d)->pW

size_t dlq_conv_packed_bytes_f8(const dlq_conv_desc* d) {
  return d && d->C > 0 && d->OC > 0 ? packed_bytes_f8(F8_GEOM(d)) : 0;
}

int dlq_pack_conv_weights_f8(const dlq_conv_desc* d, const uint8_t* q, int IC, uint8_t* packed) {
  if (!d || !q || !packed || IC <= 0 || IC > d->C || d->OC <= 0 || packed_bytes_f8(F8_GEOM(d)) == 0)
    return fail(DLQ_ERR_ARG, "pack_conv_weights_f8: unsupported shape (need C%64==0 or the 7x7 C=4 stem)");
  pack_conv_weights_f8(F8_GEOM(d), q, IC, packed);
  return DLQ_OK;
}

int dlq_conv2d_nhwc_f8(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, const float* alpha,
                       const float* beta, const uint8_t* residual, float res_scale, int relu, uint8_t* y,
                       void* stream) {
  if (!d || !alpha || !beta) return fail(DLQ_ERR_ARG, "conv2d_f8: null pointer");
  if (d->C <= 0 || d->OC <= 0 || packed_bytes_f8(F8_GEOM(d)) == 0)
    return fail(DLQ_ERR_ARG, "conv2d_f8: unsupported C (need C%64==0, or C==4 with a 7x7 kernel)");
  ConvArgs a;
  int rc = conv_args_checked(d, (const int8_t*)x, (const int8_t*)w_packed, alpha, beta, (const int8_t*)residual,
                             res_scale, relu, DLQ_OUT_S8, y, a);
  if (rc) return rc;
  if (a.P == 0) return DLQ_OK;
  const hipError_t e = f8_wide(F8_GEOM(d)) ? launch_wide_f8(a, (hipStream_t)stream)
                                           : launch_conv_f8(a, (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("conv2d_f8 launch: ") + hipGetErrorString(e));
}

int dlq_conv2d_s2_ds_nhwc_f8(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, const float* alpha,
                             const float* beta, const uint8_t* w_ds, const float* alpha_ds, const float* beta_ds,
                             uint8_t* y, uint8_t* y_ds, void* stream) {
  if (!d || !conv3x3s2_shape(F8_GEOM(d)))
    return fail(DLQ_ERR_ARG, "conv2d_s2_ds_f8: needs a 3x3/s2/p1 C->2C conv at 56x56x64, 28x28x128 or 14x14x256");
  if (!alpha || !beta || !w_ds || !alpha_ds || !beta_ds || !y_ds)
    return fail(DLQ_ERR_ARG, "conv2d_s2_ds_f8: null pointer");
  if (!f8_wide(F8_GEOM(d))) return fail(DLQ_ERR_STATE, "conv2d_s2_ds_f8: shape not supported by the fused fp8 stride-2 kernel");
  ConvArgs a;
  int rc = conv_args_checked(d, (const int8_t*)x, (const int8_t*)w_packed, alpha, beta, nullptr, 0.f, 1, DLQ_OUT_S8,
                             y, a);
  if (rc) return rc;
  if (a.P == 0) return DLQ_OK;
  const hipError_t e = launch_conv3x3s2i_f8(a, w_ds, alpha_ds, beta_ds, y_ds, (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK
                         : fail(DLQ_ERR_LAUNCH, std::string("conv2d_s2_ds_f8 launch: ") + hipGetErrorString(e));
}

int dlq_conv2d_nhwc_f8_acc(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, float* acc,
                           void* stream) {
  if (!d || d->C <= 0 || d->OC <= 0 || packed_bytes_f8(F8_GEOM(d)) == 0)
    return fail(DLQ_ERR_ARG, "conv2d_f8_acc: unsupported shape (need C%64==0, or C==4 with a 7x7 kernel)");
  ConvArgs a;
  int rc = conv_args_checked(d, (const int8_t*)x, (const int8_t*)w_packed, nullptr, nullptr, nullptr, 0.f, 0,
                             DLQ_OUT_S32, acc, a);
  if (rc) return rc;
  if (a.P == 0) return DLQ_OK;
  const hipError_t e = f8_wide(F8_GEOM(d)) ? launch_wide_f8(a, (hipStream_t)stream)
                                           : launch_conv_f8(a, (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("conv2d_f8_acc launch: ") + hipGetErrorString(e));
}

int dlq_pack_stem_weights_f8(const uint8_t* q_oihw, const float* alpha, uint8_t* packed, float* alpha_packed) {
  if (!q_oihw || !alpha || !packed || !alpha_packed) return fail(DLQ_ERR_ARG, "pack_stem_weights_f8: null");
  pack_stem_weights_f8(q_oihw, alpha, packed, alpha_packed);
  return DLQ_OK;
}

int dlq_stem_fused_f8(const float* x, int N, const uint8_t* w_stem, const float* alpha, const float* beta,
                      float inv_s, uint8_t* y, void* stream) {
  if (N < 0) return fail(DLQ_ERR_ARG, "stem_fused_f8: bad batch");
  if (N == 0) return DLQ_OK;
  if (!x || !w_stem || !alpha || !beta || !y) return fail(DLQ_ERR_ARG, "stem_fused_f8: null pointer");
  if ((long long)N * 3 * 224 * 224 * 4 >= (1LL << 31) * 4LL) return fail(DLQ_ERR_ARG, "stem_fused_f8: batch too large");
  const hipError_t e =
      launch_stem_fused(x, N, (const int8_t*)w_stem, alpha, beta, inv_s, (int8_t*)y, (hipStream_t)stream, true);
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("stem_fused_f8 launch: ") + hipGetErrorString(e));
}

int dlq_block_l1_nhwc_f8(const uint8_t* x, int N, const uint8_t* w1, const float* alpha1, const float* beta1,
                         const uint8_t* w2, const float* alpha2, const float* beta2, float s_res, uint8_t* y,
                         void* stream) {
  if (N < 0) return fail(DLQ_ERR_ARG, "block_l1_f8: bad batch");
  if (N == 0) return DLQ_OK;
  if (!x || !w1 || !alpha1 || !beta1 || !w2 || !alpha2 || !beta2 || !y)
    return fail(DLQ_ERR_ARG, "block_l1_f8: null pointer");
  const hipError_t e = launch_block_l1((const int8_t*)x, N, (const int8_t*)w1, alpha1, beta1, (const int8_t*)w2, alpha2,
                                       beta2, s_res, (int8_t*)y, (hipStream_t)stream, true);
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("block_l1_f8 launch: ") + hipGetErrorString(e));
}

int dlq_gap_nhwc_f8(const uint8_t* x, int N, int C, int HW, float k, uint8_t* y, void* stream) {
  if (N < 0 || C <= 0 || C % 4 || HW <= 0) return fail(DLQ_ERR_ARG, "gap_f8: bad shape (C % 4 == 0)");
  if (N == 0) return DLQ_OK;
  if (!x || !y) return fail(DLQ_ERR_ARG, "gap_f8: null pointer");
  if ((long long)HW * 229376 >= (1LL << 31)) return fail(DLQ_ERR_ARG, "gap_f8: HW too large for exact int32 sums");
  if (C % 16 == 0) {
    const long total = (long)N * (C / 16) * 8;
    hipLaunchKernelGGL(gap16_f8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                       N, C, HW, k, y);
  } else {
    hipLaunchKernelGGL(gap_f8_kernel, dim3(grid_for((long)N * (C / 4))), dim3(256), 0, (hipStream_t)stream, x, N, C,
                       HW, k, y);
  }
  return launch_result("gap_f8");
}

int dlq_linear_f8(const uint8_t* x, int N, int K, const uint8_t* w, int O, const float* alpha, const float* beta,
                  float* y, void* stream) {
  if (N < 0 || K <= 0 || K % 4 || O <= 0) return fail(DLQ_ERR_ARG, "linear_f8: bad shape (K % 4 == 0)");
  if (N == 0) return DLQ_OK;
  if (!x || !w || !alpha || !beta || !y) return fail(DLQ_ERR_ARG, "linear_f8: null pointer");
  if (K % 64 == 0 && !((uintptr_t)w & 15) && !((uintptr_t)x & 15)) {  // f64 MFMA kernel
    const dim3 grid((O + 63) / 64, (N + 15) / 16);
    hipLaunchKernelGGL(linear_f8_mfma_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, N, K, w, O, alpha, beta, y);
    return launch_result("linear_f8");
  }
  if ((size_t)kFcImgs * K * 4 > 64 * 1024) return fail(DLQ_ERR_ARG, "linear_f8: K too large");
  if ((uintptr_t)w & 3) return fail(DLQ_ERR_ARG, "linear_f8: misaligned weights");
  const dim3 grid((O + 255) / 256, (N + kFcImgs - 1) / kFcImgs);
  hipLaunchKernelGGL(linear_f8_kernel, grid, dim3(256), kFcImgs * K * sizeof(float), (hipStream_t)stream, x, N, K, w,
                     O, alpha, beta, y);
  return launch_result("linear_f8");
}

}  // extern "C"
