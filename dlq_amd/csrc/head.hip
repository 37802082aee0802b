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

// gap16_kernel for HW <= 8 * NPL (the ResNet-18 head: HW = 49, NPL = 7):
// the same threads, sums and requantisation, but every pixel load of a
// thread is issued before the first add, so the kernel waits for memory once
// (gap16_kernel's loop keeps two loads in flight: four round trips at HW = 49).
template <int NPL>
__global__ __launch_bounds__(256) void gap16_once_kernel(const int8_t* __restrict__ x, int N, int C, int HW, float k,
                                                         int8_t* __restrict__ y) {
  const int tpi = (C / 16) * 8;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = (int)(t / tpi), r = (int)(t - (long)n * tpi);
  const int pg = r & 7, cg = r >> 3;
  const int8_t* src = x + (size_t)(n < N ? n : 0) * HW * C + cg * 16;
  v4i v[NPL];
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    const int i = pg + 8 * j;
    v[j] = i < HW ? *(const v4i*)(src + (size_t)i * C) : v4i{0, 0, 0, 0};
  }
  int s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = 0;
#pragma unroll
  for (int j = 0; j < NPL; ++j)
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int b = 0; b < 4; ++b) s[w * 4 + b] += (int)(signed char)(v[j][w] >> (8 * b));
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

// linear_kernel<1> for K = 512 (the ResNet-18 FC on the GAP codes): the same
// tile, integers and epilogue, but every load -- the 16 k-steps' A and B
// fragments and the 16 epilogue constants of each kind -- is issued before
// the first MFMA, so the wave waits for memory once instead of once per
// four k-steps.  Two independent accumulation chains.
__global__ __launch_bounds__(64) void linear512_f32_kernel(const int8_t* __restrict__ x, int N,
                                                           const int8_t* __restrict__ w, int OC, int OCp,
                                                           const float* __restrict__ alpha,
                                                           const float* __restrict__ beta, float* __restrict__ y) {
  constexpr int K = 512, NK = K / 32;
  const int lane = threadIdx.x, lr = lane & 31, lh = lane >> 5;
  const int ot = blockIdx.x, rt = blockIdx.y;
  const int oc = ot * 32 + lr, ol = oc & 63;
  const int row = min(rt * 32 + lr, N - 1);
  const int8_t* wp = w + ((size_t)(oc >> 6) * 64 + ol) * 64;
  const size_t wstride = (size_t)(OCp / 64) * 64 * 64;
  const int sw = (ol >> 2) & 3;
  const int8_t* xp = x + (size_t)row * K + lh * 16;
  v4i a[NK], b[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    a[kk] = *(const v4i*)(wp + (size_t)(kk >> 1) * wstride + ((((2 * kk + lh) & 3) ^ sw) << 4));
    b[kk] = *(const v4i*)(xp + kk * 32);
  }
  float al[16], be[16];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = min(ot * 32 + 8 * g + 4 * lh + e, OCp - 1);  // alpha/beta are OCp long
      al[4 * g + e] = alpha[o];
      be[4 * g + e] = beta[o];
    }
  __builtin_amdgcn_sched_barrier(0);  // every load above is issued before the first MFMA
  v16i acc0 = v16i{0}, acc1 = v16i{0};
#pragma unroll
  for (int kk = 0; kk < NK; kk += 2) {
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kk], b[kk], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kk + 1], b[kk + 1], acc1, 0, 0, 0);
  }
  const v16i acc = acc0 + acc1;
  const int r = rt * 32 + lr;
  if (r >= N) return;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int o0 = ot * 32 + 8 * g + 4 * lh;
    float* dst = y + (size_t)r * OC + o0;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (o0 + e < OC) dst[e] = __builtin_fmaf((float)acc[4 * g + e], al[4 * g + e], be[4 * g + e]);
  }
}

// gap_fc_kernel: the network head (GAP + FC, RK/runtime/infer_e2e.cu:417-433)
// in ONE launch for C = K = 512, fp32 logits -- the same integers and the same
// float ops as gap16_kernel followed by linear_kernel<1>, so the logits are
// bit-identical.  Workgroup = GF images x 256 output channels, 8 waves (grid
// GF-image groups x 4: 256 workgroups at B = 256; the four workgroups of an
// image group have block ids 64 apart, i.e. the same XCD, so they share its
// L2 copy of the activations).  The head is latency-bound (6.4 MB in, 0.26
// GOP): every wave issues ALL its loads first -- its output tile's 16 weight
// fragments, the epilogue constants of its 16 outputs per lane, then its
// share of the activations -- so it waits for memory once.
//   Phase 1: wave w sums half (w & 1) of image w >> 1's pixels; lane =
//   (pixel parity, 16-channel group), one v_permlane32_swap joins the
//   parities; the halves meet as int32 partial sums in LDS, then the int8
//   GAP codes (clamp(rne(float(sum) * k))) go to LDS.
//   Phase 2: wave w runs linear_kernel's MFMA loop for output tile w of the
//   workgroup's 256 channels, B fragments from LDS (lanes lr >= GF read a
//   duplicate row; their D columns are not stored).
constexpr int GF = 4;        // images per workgroup
constexpr int GF_PL = 14;    // pixel loads per lane: HW <= 4 * GF_PL (two waves x two parities)
constexpr int GF_OCW = 256;  // output channels per workgroup (8 waves x 1 tile)

__global__ __launch_bounds__(512) void gap_fc_kernel(const int8_t* __restrict__ x, int N, int HW, float k,
                                                     const int8_t* __restrict__ w, int OC, int OCp,
                                                     const float* __restrict__ alpha, const float* __restrict__ beta,
                                                     float* __restrict__ y) {
  constexpr int C = 512, NK = C / 32;
  __shared__ __attribute__((aligned(16))) int8_t g[GF * C];
  __shared__ __attribute__((aligned(16))) int part[GF][C];  // the second half's partial sums
  __shared__ __attribute__((aligned(16))) float eab_s[2 * GF_OCW];  // alpha, beta of the workgroup's outputs
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, lr = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.x * GF;
  const size_t wstride = (size_t)(OCp / 64) * 64 * 64;
  const int ot = (blockIdx.y * GF_OCW) / 32 + wv;  // this wave's output tile
  // 1. loads in the order of need (vmcnt counts in issue order): this
  // wave's activations, the output tile's weight fragments, the epilogue
  // constants of its 16 outputs per lane
  const int img = wv >> 1, half = wv & 1, cg = lane & 31, par = lane >> 5;
  const int hh = (HW + 1) >> 1, p0 = half * hh, p1 = half ? HW : hh;  // this wave's pixels [p0, p1)
  const int n = min(n0 + img, N - 1);  // a short last group re-reads a valid image
  const int8_t* src = x + (size_t)n * HW * C + cg * 16;
  v4i v[GF_PL];
#pragma unroll
  for (int j = 0; j < GF_PL; ++j) v[j] = *(const v4i*)(src + (size_t)min(p0 + par + 2 * j, HW - 1) * C);
  v4i a0[NK];
  {
    const int oc = min(ot * 32, OCp - 32) + lr, ol = oc & 63, sw = (ol >> 2) & 3;
    const int8_t* wp = w + ((size_t)(oc >> 6) * 64 + ol) * 64;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      a0[kk] = *(const v4i*)(wp + (size_t)(kk >> 1) * wstride + ((((2 * kk + lh) & 3) ^ sw) << 4));
  }
  // the workgroup's 256 alpha / beta: one of each per thread, through LDS
  const int oe = min(blockIdx.y * GF_OCW + (t & (GF_OCW - 1)), OC - 1);
  const float eab = t < GF_OCW ? alpha[oe] : beta[oe];
  __builtin_amdgcn_sched_barrier(0);  // every load above is issued before the first sum
  int s[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) s[e] = 0;
#pragma unroll
  for (int j = 0; j < GF_PL; ++j) {
    const bool ok = p0 + par + 2 * j < p1;
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
  eab_s[t] = eab;
  if (half == 1 && par == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) *(v4i*)(&part[img][cg * 16 + 4 * q]) = v4i{s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
  }
  __syncthreads();
  if (half == 0 && par == 0) {  // exact int32 channel sums, then the GAP requantisation
    v4i o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4i pp = *(const v4i*)(&part[img][cg * 16 + 4 * q]);
      unsigned u = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) u |= ((unsigned)sat_rne((float)(s[q * 4 + b] + pp[b]) * k) & 0xffu) << (8 * b);
      o[q] = (int)u;
    }
    *(v4i*)(g + img * C + cg * 16) = o;
  }
  __syncthreads();

  // 2. FC tile ot: B fragments from LDS, two independent accumulation chains
  const int8_t* gb = g + (lr & (GF - 1)) * C + lh * 16;
  v16i acc0 = v16i{0}, acc1 = v16i{0};
#pragma unroll
  for (int kk = 0; kk < NK; kk += 2) {
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[kk], *(const v4i*)(gb + kk * 32), acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[kk + 1], *(const v4i*)(gb + (kk + 1) * 32), acc1, 0, 0, 0);
  }
  const v16i acc = acc0 + acc1;
  const int r = n0 + lr;
  if (lr >= GF || r >= N || ot * 32 >= OC) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int o0 = ot * 32 + 8 * q + 4 * lh, ol = o0 - blockIdx.y * GF_OCW;
    const v4i a4 = *(const v4i*)(eab_s + ol), b4 = *(const v4i*)(eab_s + GF_OCW + ol);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (o0 + e < OC)
        y[(size_t)r * OC + o0 + e] = __builtin_fmaf((float)acc[4 * q + e], __int_as_float(a4[e]), __int_as_float(b4[e]));
  }
}

// One-launch int8 MLP forward (the MNIST forward of CUDA/MNIST_on_GPU/v4.cu:
// 255-302 -- matmul_a_b + bias_forward + relu_forward, matmul_a_b +
// bias_forward -- and v5.cu:127-157).  The forward is 0.2 GOP: what bounds it
// is instructions and memory round trips per wave, so the grid spreads it over
// every CU (MLP_MR = 4 rows per workgroup: 256 workgroups at B = 1024, one
// wave per SIMD) and each wave waits for memory about once:
//   0. each wave issues its input-row loads, one epilogue constant of each
//      kind per thread, and the weight fragments of its first fc1 tile (all 26 k-steps of MNIST's
//      K = 832) and of its fc2 tile;
//   1. the rows -> q = clamp(rne(x * inv_s)) into LDS (quantize_rows_kernel's
//      op sequence; zeros beyond `in`);
//   2. fc1 on v_mfma_i32_32x32x32_i8 (A = 32 hidden units of the packed
//      weights, B = the LDS rows, lane l reading row l & 3), epilogue
//      fmaf(acc, a1, b1), ReLU, requant into LDS (and the global hidden buffer
//      dlq_mlp_copy_hidden reads);
//   3. fc2 from LDS, epilogue fmaf(acc, a2, b2) -> fp32 logits.
// Per element the same integer sums and IEEE ops as quantize_rows_kernel +
// linear_kernel<0> + linear_kernel<1>: bit-identical to the three-launch
// forward.  Every load reads a valid (clamped) address outside any branch (a
// load on one side of a branch costs a vmcnt(0) at the join); values past the
// ends are never used.
#ifdef DLQ_STAMPS
__device__ unsigned long long g_mlp_stamps[1024 * 4 * 8];
#define MSTAMP(i)                                                                                            \
  do {                                                                                                       \
    if ((threadIdx.x & 63) == 0) g_mlp_stamps[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define MSTAMP(i) \
  do {            \
  } while (0)
#endif
constexpr int MLP_NW = 4;   // waves
constexpr int MLP_MR_DEFAULT = 4;
constexpr int MLP_KB = 26;  // fc1 k-steps per register batch (K = 832)
// fc2 k-steps prefetched at kernel start: the kernel's W2 template argument,
// H / 32 for H <= 128 (MNIST: 4 -- loading 8 re-read the last fragment four
// times per wave) and 8 above

// The fused kernel's weight images are fragment-major (mlp.cpp
// mlp_fragment_image): fragment (k-step k, 32-channel tile t) is 1 KiB at
// (k * T + t) * 1024, lane l's 16 bytes at l * 16, so every fragment load of
// a wave reads one contiguous KiB (the generic packed image spread it over
// 32 rows: 4x the cache lines per load, and loading the weights was the
// launch's longest phase).
__device__ __forceinline__ v4i mlp_frag(const int8_t* wf, int T, int k, int t, int lane) {
  return *(const v4i*)(wf + ((size_t)k * T + t) * 1024 + lane * 16);
}
template <int NF>
__device__ __forceinline__ void mlp_frags(const int8_t* wf, int T, int kb, int nk, int t, int lane, v4i (&f)[NF]) {
#pragma unroll
  for (int i = 0; i < NF; ++i) f[i] = mlp_frag(wf, T, kb + i < nk ? kb + i : nk - 1, t, lane);  // never past the last
}

template <int MLP_MR, int MLP_W2>  // rows per workgroup (= input float4 loads per thread issued up front)
__global__ __launch_bounds__(MLP_NW * 64) void mlp_fused_kernel(
    const float* __restrict__ x, int N, int in, int kp, float inv_s, const int8_t* __restrict__ w1, int H,
    int OCp1, const float* __restrict__ a1, const float* __restrict__ b1, const int8_t* __restrict__ w2, int OC,
    int OCp2, const float* __restrict__ a2, const float* __restrict__ b2, int8_t* __restrict__ hq_g,
    float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) int8_t mlp_lds[];
  const int xp = kp + 16, hp = H + 16;
  int8_t* xq = mlp_lds;
  int8_t* hq = xq + MLP_MR * xp;
  float* ab = (float*)(hq + MLP_MR * hp);  // a1[H] b1[H] a2[OCp2] b2[OCp2]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int r0 = blockIdx.x * MLP_MR, br = lr & (MLP_MR - 1), nrow = min(MLP_MR, N - r0);
  const int T = H / 32, T2 = (OC + 31) / 32, nk1 = kp / 32, nk2 = H / 32, u4 = kp >> 2;
  const int TI1 = OCp1 / 32, TI2 = OCp2 / 32;  // tiles per k-step in the fragment images
  MSTAMP(0);

  // 0. loads, in the order of need (vmcnt counts in issue order)
  const bool vec = (in & 3) == 0 && u4 <= MLP_NW * 64;  // one float4 per thread and row (MNIST: 196 per row)
  float4 f[MLP_MR];
  if (vec) {
    const unsigned xo = (unsigned)min(4 * tid, in - 4) * 4u;
#pragma unroll
    for (int r = 0; r < MLP_MR; ++r)
      f[r] = *(const float4*)((const char*)(x + (size_t)(r0 + min(r, nrow - 1)) * in) + xo);
  }
  const int t1 = min(wave, T - 1), t2 = min(wave, T2 - 1);  // this wave's first fc1 / fc2 tiles
  // epilogue constants, one of each per thread (to LDS after the quantisation)
  const float ca1 = a1[min(tid, H - 1)], cb1 = b1[min(tid, H - 1)];
  const float ca2 = a2[min(tid, OC - 1)], cb2 = b2[min(tid, OC - 1)];
  v4i fa[MLP_KB];
  mlp_frags(w1, TI1, 0, nk1, t1, lane, fa);
  v4i f2[MLP_W2];
  mlp_frags(w2, TI2, 0, nk2, t2, lane, f2);
  MSTAMP(1);

  // 1. quantise the rows into LDS
  auto quant = [&](float v0, float v1, float v2, float v3) -> unsigned {
    return ((unsigned)sat_rne(v0 * inv_s) & 0xffu) | (((unsigned)sat_rne(v1 * inv_s) & 0xffu) << 8) |
           (((unsigned)sat_rne(v2 * inv_s) & 0xffu) << 16) | (((unsigned)sat_rne(v3 * inv_s) & 0xffu) << 24);
  };
  if (vec) {
#pragma unroll
    for (int r = 0; r < MLP_MR; ++r) {
      const bool ok = r < nrow && 4 * tid < in;
      if (tid < u4)
        *(unsigned*)(xq + r * xp + 4 * tid) =
            quant(ok ? f[r].x : 0.f, ok ? f[r].y : 0.f, ok ? f[r].z : 0.f, ok ? f[r].w : 0.f);
    }
  } else {
    for (int u = tid; u < MLP_MR * u4; u += MLP_NW * 64) {
      const int r = u / u4, c0 = 4 * (u - r * u4), row = r0 + r;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = row < N && c0 + e < in ? x[(size_t)row * in + c0 + e] : 0.f;
      *(unsigned*)(xq + r * xp + c0) = quant(v[0], v[1], v[2], v[3]);
    }
  }
  if (tid < H) {
    ab[tid] = ca1;
    ab[H + tid] = cb1;
  }
  if (tid < OC) {
    ab[2 * H + tid] = ca2;
    ab[2 * H + OCp2 + tid] = cb2;
  }
  for (int i = MLP_NW * 64 + tid; i < H; i += MLP_NW * 64) {
    ab[i] = a1[i];
    ab[H + i] = b1[i];
  }
  for (int i = MLP_NW * 64 + tid; i < OC; i += MLP_NW * 64) {
    ab[2 * H + i] = a2[i];
    ab[2 * H + OCp2 + i] = b2[i];
  }
  __syncthreads();
  MSTAMP(2);

  // 2. fc1 + bias + ReLU + requant: tiles wave, wave + 4, ...
  for (int ot = wave; ot < T; ot += MLP_NW) {
    // k-steps mod 4: four independent MFMA chains (a dependent chain pays the
    // MFMA's latency per step; this launch is latency-bound), summed (exact int32)
    v16i ac4[4] = {v16i{0}, v16i{0}, v16i{0}, v16i{0}};
    for (int kb = 0; kb < nk1; kb += MLP_KB) {
      if (kb > 0 || ot != wave) mlp_frags(w1, TI1, kb, nk1, ot, lane, fa);
#pragma unroll
      for (int i = 0; i < MLP_KB; ++i)
        if (kb + i < nk1) {  // wave-uniform
          const v4i bf = *(const v4i*)(xq + br * xp + (kb + i) * 32 + lh * 16);
          ac4[i & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], bf, ac4[i & 3], 0, 0, 0);
        }
    }
    const v16i acc = (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
    if (lr < MLP_MR) {  // D column lr = row r0 + lr
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int o0 = ot * 32 + 8 * g + 4 * lh;
        const v4i al = *(const v4i*)(ab + o0), be = *(const v4i*)(ab + H + o0);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf((float)acc[4 * g + e], __int_as_float(al[e]), __int_as_float(be[e]));
        const unsigned q = quant4(v[0], v[1], v[2], v[3], 0.f);
        *(unsigned*)(hq + lr * hp + o0) = q;
        if (lr < nrow) *(unsigned*)(hq_g + (size_t)(r0 + lr) * H + o0) = q;
      }
    }
  }
  __syncthreads();
  MSTAMP(3);

  // 3. fc2 + bias -> fp32 logits
  for (int ot = wave; ot < T2; ot += MLP_NW) {
    v16i acc = v16i{0};
#pragma unroll
    for (int k = 0; k < MLP_W2; ++k)
      if (k < nk2) {
        const v4i a = ot == wave ? f2[k] : mlp_frag(w2, TI2, k, ot, lane);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, *(const v4i*)(hq + br * hp + k * 32 + lh * 16), acc, 0, 0, 0);
      }
    for (int k = MLP_W2; k < nk2; ++k)
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(mlp_frag(w2, TI2, k, ot, lane),
                                                  *(const v4i*)(hq + br * hp + k * 32 + lh * 16), acc, 0, 0, 0);
    if (lr < nrow) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int o0 = ot * 32 + 8 * g + 4 * lh;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (o0 + e < OC)
            y[(size_t)(r0 + lr) * OC + o0 + e] =
                __builtin_fmaf((float)acc[4 * g + e], ab[2 * H + o0 + e], ab[2 * H + OCp2 + o0 + e]);
      }
    }
  }
  MSTAMP(4);
}

}  // namespace

// The fused MNIST forward: kp % 64 == 0, kp >= in, H % 64 == 0.
template <int MR>
size_t mlp_lds_bytes(int kp, int H, int OC) {
  return (size_t)MR * (kp + 16) + (size_t)MR * (H + 16) + (size_t)(2 * H + 2 * packed_oc(OC)) * 4;
}

// The fused kernel's dynamic LDS must fit the 64 KiB it is launched with.
bool mlp_fused_fits(int kp, int H, int OC, int mr) {
  if (mr == 0) mr = MLP_MR_DEFAULT;
  const size_t lds = mr == 16 ? mlp_lds_bytes<16>(kp, H, OC)
                     : mr == 8 ? mlp_lds_bytes<8>(kp, H, OC)
                               : mlp_lds_bytes<4>(kp, H, OC);
  return lds <= 64 * 1024;
}

template <int MR>
hipError_t launch_mlp_mr(const float* x, int N, int in, int kp, float inv_s, const int8_t* w1, int H,
                         const float* a1, const float* b1, const int8_t* w2, int OC, const float* a2,
                         const float* b2, int8_t* hq, float* y, hipStream_t s) {
  const size_t lds = mlp_lds_bytes<MR>(kp, H, OC);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
if (H <= 64)
    hipLaunchKernelGGL((mlp_fused_kernel<MR, 2>), dim3((N + MR - 1) / MR), dim3(MLP_NW * 64), lds, s, x, N, in, kp,
                       inv_s, w1, H, packed_oc(H), a1, b1, w2, OC, packed_oc(OC), a2, b2, hq, y);
  else if (H <= 128)
    hipLaunchKernelGGL((mlp_fused_kernel<MR, 4>), dim3((N + MR - 1) / MR), dim3(MLP_NW * 64), lds, s, x, N, in, kp,
                       inv_s, w1, H, packed_oc(H), a1, b1, w2, OC, packed_oc(OC), a2, b2, hq, y);
  else
    hipLaunchKernelGGL((mlp_fused_kernel<MR, 8>), dim3((N + MR - 1) / MR), dim3(MLP_NW * 64), lds, s, x, N, in, kp,
                       inv_s, w1, H, packed_oc(H), a1, b1, w2, OC, packed_oc(OC), a2, b2, hq, y);
  return hipGetLastError();
}

// The fused MNIST forward: kp % 64 == 0, kp >= in, H % 64 == 0.  mr = rows
// per workgroup (4, 8 or 16; 0 = the default for N).
hipError_t launch_mlp_fused(const float* x, int N, int in, int kp, float inv_s, const int8_t* w1, int H,
                            const float* a1, const float* b1, const int8_t* w2, int OC, const float* a2,
                            const float* b2, int8_t* hq, float* y, hipStream_t s, int mr) {
  if (N < 1 || in < 1 || kp % 64 || kp < in || H < 64 || H % 64 || OC < 1) return hipErrorInvalidValue;
  if (mr == 0) mr = MLP_MR_DEFAULT;
  if (mr == 4) return launch_mlp_mr<4>(x, N, in, kp, inv_s, w1, H, a1, b1, w2, OC, a2, b2, hq, y, s);
  if (mr == 8) return launch_mlp_mr<8>(x, N, in, kp, inv_s, w1, H, a1, b1, w2, OC, a2, b2, hq, y, s);
  if (mr == 16) return launch_mlp_mr<16>(x, N, in, kp, inv_s, w1, H, a1, b1, w2, OC, a2, b2, hq, y, s);
  return hipErrorInvalidValue;
}

// C = K = 512, HW <= 56 (the ResNet-18 head); hipErrorInvalidValue otherwise.
hipError_t launch_gap_fc(const int8_t* x, int N, int C, int HW, float k, const int8_t* w, int OC,
                         const float* alpha, const float* beta, float* y, hipStream_t s) {
  if (C != 512 || HW < 1 || HW > 4 * GF_PL || N < 1 || OC < 1) return hipErrorInvalidValue;
  const int OCp = packed_oc(OC);
  const dim3 grid((N + GF - 1) / GF, (OC + GF_OCW - 1) / GF_OCW);
  hipLaunchKernelGGL(gap_fc_kernel, grid, dim3(512), 0, s, x, N, HW, k, w, OC, OCp, alpha, beta, y);
  return hipGetLastError();
}

hipError_t launch_gap(const int8_t* x, int N, int C, int HW, float k, int8_t* y, hipStream_t s) {
  const long total = (long)N * (C / 16) * 8;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (HW <= 8)
    hipLaunchKernelGGL(gap16_once_kernel<1>, grid, block, 0, s, x, N, C, HW, k, y);
  else if (HW <= 56)
    hipLaunchKernelGGL(gap16_once_kernel<7>, grid, block, 0, s, x, N, C, HW, k, y);
  else
    hipLaunchKernelGGL(gap16_kernel, grid, block, 0, s, x, N, C, HW, k, y);
  return hipGetLastError();
}

hipError_t launch_linear(const int8_t* x, int N, int K, const int8_t* w, int OC, const float* alpha,
                         const float* beta, int relu, int out_kind, void* y, hipStream_t s) {
  const int OCp = packed_oc(OC);
  const dim3 grid((OC + 31) / 32, (N + 31) / 32), block(64);
  if (out_kind == 1 && K == 512)
    hipLaunchKernelGGL(linear512_f32_kernel, grid, block, 0, s, x, N, w, OC, OCp, alpha, beta, (float*)y);
  else if (out_kind == 1)
    hipLaunchKernelGGL(linear_kernel<1>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  else if (out_kind == 2)
    hipLaunchKernelGGL(linear_kernel<2>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  else
    hipLaunchKernelGGL(linear_kernel<0>, grid, block, 0, s, x, N, K, w, OC, OCp, alpha, beta, relu, y);
  return hipGetLastError();
}

}  // namespace dlq
