// ref_f32.hip -- the reference's fp32 ResNet-18 semantics on the GPU, op for
// op, for activation-scale calibration and the launcher's fp32 mode.
//
// This is NOT the hot path (the int8 engine is): it is model preparation and a
// parity tool.  Each kernel repeats one reference kernel's arithmetic exactly
// (RK = CUDA/resnet18-kernel-lab/cpp/fp32):
//   conv   im2col (RK/kernels/im2col.cu:37-54, rows r = c*kH*kW + kh*kW + kw,
//          zero padding) + sgemm_tiled (sgemm_tiled.cu:22-45): every output is
//          acc = fmaf(w[oc][r], col[r][p], acc) over r = 0..K-1 in order, the
//          padding zeros included (nvcc contracts `acc += a*b`);
//   bn     bn_inference.cu:22-27: y = fmaf(g, (x - m) / sqrtf(v + eps), b);
//   relu   relu.cu:9; add add.cu:7 (y += x); maxpool maxpool2d.cu:14-40;
//   gap    gap_global_ref (RK/runtime/infer_e2e.cu:37-61): 256 strided partial
//          sums, a tree over strides 128..1, then / HW;
//   fc     fc_forward (:206-219): the same fmaf GEMM (N = 1) + fp32 bias add.
// so the results are bit-identical to oracle.c's ora_*_f32, which the
// reference's golden vector out/step8_logits.bin pins.  One thread per output
// element: a few ms per image, run once per calibration.
//
// Site amax: max |v| over a tensor, as the uint bit pattern of fabsf(v) (for
// non-negative floats bit order is value order), wave-reduced then at most one
// atomicMax per wave.
#include <cfloat>

#include "device_common.h"

namespace dlq {
namespace {

__device__ __forceinline__ void amax_update(unsigned* amax, float v) {
  if (!amax) return;
  unsigned u = __float_as_uint(fabsf(v));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned t = (unsigned)__shfl_xor((int)u, o, 64);
    u = t > u ? t : u;
  }
  // skip the atomic when the site's running max already covers the wave's:
  // the max only grows, so a stale read only costs an unneeded atomic (one
  // atomic per wave on one address serialised the 6.4M-element residual adds
  // of a 32-image calibration at ~0.5 ms each)
  if ((threadIdx.x & 63) == 0 && u > __hip_atomic_load(amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(amax, u);
}

// y[n][oc][oh][ow] = bn(conv(x))[, relu]; d[oc] = sqrtf(var + eps) (host-computed, IEEE).
__global__ __launch_bounds__(256) void ref_conv_bn_kernel(const float* __restrict__ x, int B, int IC, int H, int W,
                                                          const float* __restrict__ w, int OC, int k, int s, int p,
                                                          const float* __restrict__ g, const float* __restrict__ bb,
                                                          const float* __restrict__ m, const float* __restrict__ d,
                                                          int relu, float* __restrict__ y, unsigned* amax) {
  const int OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  const long total = (long)B * OC * OH * OW;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (i < total) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH), oc = (int)((i / ((long)OW * OH)) % OC);
    const int n = (int)(i / ((long)OW * OH * OC));
    const float* xn = x + (size_t)n * IC * H * W;
    const float* wr = w + (size_t)oc * IC * k * k;
    float acc = 0.f;
    for (int c = 0; c < IC; ++c)
      for (int kh = 0; kh < k; ++kh) {
        const int ih = oh * s - p + kh;
        for (int kw = 0; kw < k; ++kw) {
          const int iw = ow * s - p + kw;
          const float xv = (ih >= 0 && iw >= 0 && ih < H && iw < W) ? xn[((size_t)c * H + ih) * W + iw] : 0.f;
          acc = __builtin_fmaf(wr[(c * k + kh) * k + kw], xv, acc);
        }
      }
    v = __builtin_fmaf(g[oc], __fdiv_rn(acc - m[oc], d[oc]), bb[oc]);
    if (relu && v < 0.f) v = 0.f;
    y[i] = v;
  }
  amax_update(amax, v);
}

// y += skip (add.cu:7); relu (relu.cu:9)
__global__ __launch_bounds__(256) void ref_add_relu_kernel(float* __restrict__ y, const float* __restrict__ skip,
                                                           long n, unsigned* amax) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (i < n) {
    v = y[i] + skip[i];
    if (v < 0.f) v = 0.f;
    y[i] = v;
  }
  amax_update(amax, v);
}

__global__ __launch_bounds__(256) void ref_maxpool_kernel(const float* __restrict__ x, int NC, int H, int W,
                                                          float* __restrict__ y) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)NC * OH * OW) return;
  const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
  const long nc = i / ((long)OW * OH);
  float vmax = -FLT_MAX;
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = oh * 2 - 1 + kh;
    if (ih < 0 || ih >= H) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int iw = ow * 2 - 1 + kw;
      if (iw < 0 || iw >= W) continue;
      const float v = x[(size_t)nc * H * W + (size_t)ih * W + iw];
      vmax = v > vmax ? v : vmax;
    }
  }
  y[i] = vmax;
}

// one 256-thread workgroup per (n, c): gap_global_ref's order
__global__ __launch_bounds__(256) void ref_gap_kernel(const float* __restrict__ x, int HW, float* __restrict__ y,
                                                      unsigned* amax) {
  __shared__ float s[256];
  const int t = threadIdx.x;
  const float* xc = x + (size_t)blockIdx.x * HW;
  float acc = 0.f;
  for (int i = t; i < HW; i += 256) acc += xc[i];
  s[t] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (t < st) s[t] += s[t + st];
    __syncthreads();
  }
  float v = 0.f;
  if (t == 0) {
    v = __fdiv_rn(s[0], (float)HW);
    y[blockIdx.x] = v;
  }
  if (t < 64) amax_update(amax, v);
}

// out[n][o] = (fmaf chain over i of W[o][i] * g[n][i]) + bias[o]
__global__ __launch_bounds__(256) void ref_fc_kernel(const float* __restrict__ g, int B, const float* __restrict__ Wt,
                                                     const float* __restrict__ bias, int O, int I,
                                                     float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * O) return;
  const int n = i / O, o = i - n * O;
  float acc = 0.f;
  for (int k = 0; k < I; ++k) acc = __builtin_fmaf(Wt[(size_t)o * I + k], g[(size_t)n * I + k], acc);
  out[i] = acc + bias[o];
}

__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long n, unsigned* amax) {
  float v = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float a = fabsf(x[i]);
    v = a > v ? a : v;
  }
  amax_update(amax, v);
}

unsigned blocks_for(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

hipError_t launch_ref_conv_bn(const float* x, int B, int IC, int H, int W, const float* w, int OC, int k, int s, int p,
                              const float* g, const float* b, const float* m, const float* d, int relu, float* y,
                              unsigned* amax, hipStream_t st) {
  const long total = (long)B * OC * ((H + 2 * p - k) / s + 1) * ((W + 2 * p - k) / s + 1);
  hipLaunchKernelGGL(ref_conv_bn_kernel, dim3(blocks_for(total)), dim3(256), 0, st, x, B, IC, H, W, w, OC, k, s, p, g,
                     b, m, d, relu, y, amax);
  return hipGetLastError();
}

hipError_t launch_ref_add_relu(float* y, const float* skip, long n, unsigned* amax, hipStream_t st) {
  hipLaunchKernelGGL(ref_add_relu_kernel, dim3(blocks_for(n)), dim3(256), 0, st, y, skip, n, amax);
  return hipGetLastError();
}

hipError_t launch_ref_maxpool(const float* x, int NC, int H, int W, float* y, hipStream_t st) {
  const long total = (long)NC * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  hipLaunchKernelGGL(ref_maxpool_kernel, dim3(blocks_for(total)), dim3(256), 0, st, x, NC, H, W, y);
  return hipGetLastError();
}

hipError_t launch_ref_gap(const float* x, int NC, int HW, float* y, unsigned* amax, hipStream_t st) {
  hipLaunchKernelGGL(ref_gap_kernel, dim3(NC), dim3(256), 0, st, x, HW, y, amax);
  return hipGetLastError();
}

hipError_t launch_ref_fc(const float* g, int B, const float* W, const float* bias, int O, int I, float* out,
                         hipStream_t st) {
  hipLaunchKernelGGL(ref_fc_kernel, dim3(blocks_for((long)B * O)), dim3(256), 0, st, g, B, W, bias, O, I, out);
  return hipGetLastError();
}

hipError_t launch_amax(const float* x, long n, unsigned* amax, hipStream_t st) {
  long g = blocks_for(n);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)g), dim3(256), 0, st, x, n, amax);
  return hipGetLastError();
}

}  // namespace dlq
