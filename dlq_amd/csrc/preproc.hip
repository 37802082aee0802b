// preproc.hip -- the two ends of the inference path around the int8 network:
//
// * image preprocessing on the device: u8 HWC RGB
//   images -> resize shorter side to 256 (PIL BILINEAR) -> centre crop 224 ->
//   /255 -> (x - mean) / std -> fp32 NCHW, the network's input
//   (RK/tools/preprocess_to_bin.py:8-33, RK = CUDA/resnet18-kernel-lab; the
//   reference runs it offline in Python and uploads the .bin,
//   RK/runtime/infer_e2e.cu:255-256).  The resize is Pillow's 8-bit
//   resampler (Resample.c: precompute_coeffs / normalize_coeffs_8bpc /
//   ImagingResampleHorizontal_8bpc / _Vertical_8bpc): triangle filter with
//   support scaled by the downscale factor, double-precision coefficients
//   normalised per output pixel and rounded to 22-bit fixed point,
//   horizontal pass first with a clip8 round trip, then vertical.  Each
//   thread computes its own coefficients in double (only +,-,*,/ and
//   truncating casts: the same IEEE results as the host) for one output
//   pixel of the crop, so no coefficient tables are needed.
//
// * the head after the logits: softmax_1d (RK/kernels/softmax.cu:5-47) per
//   row and the launcher's top-1 (RK/runtime/infer_e2e.cu:436-438, first
//   index with logit > the running best, starting from -1e30), one wave per
//   row with xor-shuffle reductions.
#include <cmath>

#include "../../include/dlq.h"
#include "device_common.h"

namespace dlq {
namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;  // Pillow Resample.c PRECISION_BITS

struct Taps {
  int lo, n;  // first source index, tap count
};

// precompute_coeffs for one output index (box = (0, in_size), bilinear
// support 1), normalised and converted like normalize_coeffs_8bpc.
__device__ __forceinline__ Taps bilinear_taps(int out_idx, int in_size, int out_size, int* k, int kmax) {
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = (out_idx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > kmax) xmax = kmax;  // never for scales this path admits (host check)
  double w[16];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    const double f = t < 1.0 ? 1.0 - t : 0.0;
    w[x] = f;
    ww += f;
  }
  for (int x = 0; x < xmax; ++x) {
    const double kx = ww != 0.0 ? w[x] / ww : w[x];
    k[x] = kx < 0 ? (int)(-0.5 + kx * (1 << kPrecisionBits)) : (int)(0.5 + kx * (1 << kPrecisionBits));
  }
  return Taps{xmin, xmax};
}

__device__ __forceinline__ int clip8(int v) {
  if (v >= (1 << kPrecisionBits) << 8) return 255;
  if (v <= 0) return 0;
  return v >> kPrecisionBits;
}

// One thread per output pixel of the 224x224 crop (all three channels).
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ img, int N, int H, int W,
                                                         int new_h, int new_w, int top, int left, int S,
                                                         float* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)S * S;
  if (t >= (long)N * per) return;
  const int n = (int)(t / per), r = (int)(t - (long)n * per), y = r / S, x = r - y * S;
  const uint8_t* src = img + (size_t)n * H * W * 3;
  const bool need_h = new_w != W, need_v = new_h != H;
  int kx[16], ky[16];
  const Taps th = need_h ? bilinear_taps(left + x, W, new_w, kx, 16) : Taps{left + x, 1};
  const Taps tv = need_v ? bilinear_taps(top + y, H, new_h, ky, 16) : Taps{top + y, 1};
  int acc[3] = {1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1)};
  int px[3] = {0, 0, 0};
  for (int j = 0; j < tv.n; ++j) {
    const uint8_t* row = src + (size_t)(tv.lo + j) * W * 3;
    int h[3];
    if (need_h) {
      int s[3] = {1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1)};
      for (int i = 0; i < th.n; ++i) {
        const uint8_t* p = row + (size_t)(th.lo + i) * 3;
        s[0] += (int)p[0] * kx[i];
        s[1] += (int)p[1] * kx[i];
        s[2] += (int)p[2] * kx[i];
      }
      h[0] = clip8(s[0]);
      h[1] = clip8(s[1]);
      h[2] = clip8(s[2]);
    } else {
      const uint8_t* p = row + (size_t)th.lo * 3;
      h[0] = p[0];
      h[1] = p[1];
      h[2] = p[2];
    }
    if (need_v) {
      acc[0] += h[0] * ky[j];
      acc[1] += h[1] * ky[j];
      acc[2] += h[2] * ky[j];
    } else {
      px[0] = h[0];
      px[1] = h[1];
      px[2] = h[2];
    }
  }
  if (need_v) {
    px[0] = clip8(acc[0]);
    px[1] = clip8(acc[1]);
    px[2] = clip8(acc[2]);
  }
  // np.float32 pixel / 255.0, then (x - mean) / std in float32 (IEEE divisions)
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = __fdiv_rn((float)px[c], 255.0f);
    out[(((size_t)n * 3 + c) * S + y) * S + x] = __fdiv_rn(v - mean[c], stdv[c]);
  }
}

// One wave per row: softmax (optional) and top-1 (optional).
__global__ __launch_bounds__(256) void softmax_top1_kernel(const float* __restrict__ x, int N, int K,
                                                           float* __restrict__ y, int* __restrict__ idx,
                                                           float* __restrict__ val) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* xr = x + (size_t)row * K;
  float mx = -INFINITY, best = -1e30f;
  int bi = 0x7fffffff;
  for (int i = lane; i < K; i += 64) {
    const float v = xr[i];
    mx = fmaxf(mx, v);
    if (v > best) {  // ascending i per lane: the first maximum of this lane
      best = v;
      bi = i;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, off));
    const float ob = __shfl_xor(best, off);
    const int oi = __shfl_xor(bi, off);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) {
    if (idx) idx[row] = bi == 0x7fffffff ? -1 : bi;
    if (val) val[row] = best;
  }
  if (!y) return;
  float s = 0.f;
  for (int i = lane; i < K; i += 64) s += expf(xr[i] - mx);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  for (int i = lane; i < K; i += 64) y[(size_t)row * K + i] = expf(xr[i] - mx) / s;
}

// Python's round() of h * size / w (half to even), as preprocess_to_bin.py:8-16.
int round_half_even(double v) { return (int)std::nearbyint(v); }

}  // namespace
}  // namespace dlq

using namespace dlq;

extern "C" {

int dlq_preprocess_size(int H, int W, int* new_h, int* new_w) {
  if (H <= 0 || W <= 0 || !new_h || !new_w) return fail(DLQ_ERR_ARG, "preprocess_size: bad args");
  if (W < H) {
    *new_w = 256;
    *new_h = round_half_even((double)H * 256 / W);
  } else {
    *new_h = 256;
    *new_w = round_half_even((double)W * 256 / H);
  }
  return DLQ_OK;
}

int dlq_preprocess_u8(const uint8_t* img, int N, int H, int W, float* out, void* stream) {
  if (N < 0 || H <= 0 || W <= 0) return fail(DLQ_ERR_ARG, "preprocess: bad shape");
  if (N == 0) return DLQ_OK;
  if (!img || !out) return fail(DLQ_ERR_ARG, "preprocess: null pointer");
  int nh, nw;
  dlq_preprocess_size(H, W, &nh, &nw);
  const int S = 224;
  if (nh < S || nw < S) return fail(DLQ_ERR_ARG, "preprocess: resized image smaller than the crop");
  // bilinear support = max(1, in/out) source pixels each side: at most 16 taps
  if ((double)H / nh > 7.0 || (double)W / nw > 7.0)
    return fail(DLQ_ERR_ARG, "preprocess: downscale factor above 7 (more than 16 filter taps)");
  if ((long long)N * H * W * 3 >= (1LL << 40)) return fail(DLQ_ERR_ARG, "preprocess: input too large");
  const int top = (nh - S) / 2, left = (nw - S) / 2;
  const long total = (long)N * S * S;
  hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     img, N, H, W, nh, nw, top, left, S, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("preprocess: ") + hipGetErrorString(e));
}

int dlq_softmax_f32(const float* x, int N, int K, float* y, void* stream) {
  if (N < 0 || K <= 0) return fail(DLQ_ERR_ARG, "softmax: bad shape");
  if (N == 0) return DLQ_OK;
  if (!x || !y) return fail(DLQ_ERR_ARG, "softmax: null pointer");
  hipLaunchKernelGGL(softmax_top1_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, N, K,
                     y, nullptr, nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("softmax: ") + hipGetErrorString(e));
}

int dlq_top1_f32(const float* x, int N, int K, int* idx, float* val, void* stream) {
  if (N < 0 || K <= 0) return fail(DLQ_ERR_ARG, "top1: bad shape");
  if (N == 0) return DLQ_OK;
  if (!x || !idx) return fail(DLQ_ERR_ARG, "top1: null pointer");
  hipLaunchKernelGGL(softmax_top1_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, N, K,
                     nullptr, idx, val);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DLQ_OK : fail(DLQ_ERR_LAUNCH, std::string("top1: ") + hipGetErrorString(e));
}

}  // extern "C"
