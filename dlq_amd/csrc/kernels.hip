// kernels.hip -- hand-written gfx950 (CDNA4) kernels of the int8 inference path.
//
//  conv_s8_kernel   implicit-im2col int8 conv / dense layer on
//                   v_mfma_i32_32x32x32_i8 with the dequant*BN, residual, ReLU
//                   and requant epilogue fused in.  Replaces im2col_nchw +
//                   sgemm_tiled + bn_inference + add_inplace + relu_forward
//                   (CUDA/resnet18-kernel-lab/cpp/fp32/kernels/{im2col,sgemm_tiled,
//                   bn_inference,add,relu}.cu) and the MNIST forward GEMMs
//                   (CUDA/MNIST_on_GPU/v4.cu:121-132,163-179).
//  quantize_*       fp32 -> int8 (HBM-bound)
//  maxpool_*        3x3/s2/p1 on int8 NHWC (kernels/maxpool2d.cu:4-41)
//  gap_*            global average pool, int32 sum + requant (infer_e2e.cu:37-61)
//  im2col_nchw_s8   reference-order im2col (kernels/im2col.cu:5-58), parity only
//
// GEMM orientation: D[oc][pixel] = sum_k W[oc][k] * X[pixel][k].  Both
// operands are K-contiguous in HBM (weights packed [OCp][K], activations NHWC
// with K ordered (kh, kw, c)), so every staging load is a 16-byte vector and
// every LDS fragment read is one ds_read_b128.  int32 sums are order
// independent, so the (kh,kw,c) K order gives the same accumulators as the
// reference's (c,kh,kw) im2col order (checked in tests/test_gpu_parity.py).
//
// MFMA lane maps (verified on gfx950 by tools/probe/mfma_i8_probe.hip):
//   A: lane l holds W[row l&31][k 16*(l>>5) .. +15]
//   B: lane l holds X[col l&31][k 16*(l>>5) .. +15]
//   D: reg r of lane l is D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
#include <cstdlib>
#include <type_traits>

#include "device_common.h"

namespace dlq {
namespace {

template <int TOC, int TP, int WOC>
struct TileCfg {
  static constexpr int WPN = 4 / WOC;           // waves along pixels
  static constexpr int WTOC = TOC / WOC;        // oc rows per wave
  static constexpr int WTP = TP / WPN;          // pixels per wave
  static constexpr int FM = WTOC / 32;          // 32x32 MFMA tiles per wave (oc)
  static constexpr int FN = WTP / 32;           // 32x32 MFMA tiles per wave (pixel)
  static constexpr int ALD = TOC * 4 / NT;      // 16-B weight chunks per thread per step
  static constexpr int BLD = TP * 4 / NT;       // 16-B activation chunks per thread per step
  static constexpr int BUF = (TOC + TP) * BK;   // bytes of one LDS stage
  static_assert(WOC * WPN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1 && ALD >= 1 && BLD >= 1, "tile too small");
};

// MODE 0: C % 64 == 0, K = kH*kW*C ordered (kh, kw, c); one K step = one
//         (kh, kw) tap and 64 channels -> one 16-B load per chunk.
// MODE 1: RGB stem, C == 4 (NHWC4, channel 3 zero), 7x7 taps padded to 8x8:
//         K = 256 ordered (kh, kw, c); one K step = 2 kh rows x 8 kw x 4 c;
//         a 16-B chunk = 4 taps of one row, loaded as 4 dwords.
// OUT: DLQ_OUT_S8 (0), DLQ_OUT_F32 (1), DLQ_OUT_S32 (2).
// F8: operands are e4m3 codes (the fp8 path): the same bytes
//     staged the same way, but each K step is ONE v_mfma_f32_32x32x64_f8f6f4
//     (the scaled builtin with zero scales lowers to the unscaled opcode) on
//     fp32 accumulators; lane half h feeds chunks h and 2+h of the step as
//     bytes 0-15 / 16-31 of its 32-byte fragment, identically for A and B, so
//     every product pairs the same k.  Epilogue enc4_f8 (OUT 0 only).
template <int TOC, int TP, int WOC, int MODE, int OUT, bool RES, bool F8 = false>
__global__ __launch_bounds__(NT) void conv_s8_kernel(ConvArgs a) {
  static_assert(!F8 || OUT != 1, "fp8 convs produce e4m3 or raw fp32 accumulators");
  using T = TileCfg<TOC, TP, WOC>;
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * T::BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wo = wave % WOC, wp = wave / WOC;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n_oc = a.OCp / TOC;
  const int oc0 = (bid % n_oc) * TOC;
  const int p0 = (bid / n_oc) * TP;

  const int H = a.H, W = a.W, C = a.C, K = a.K;
  const int srow = tid >> 2, sch = tid & 3;  // staging row / chunk of this thread

  // Per staging slot: base pixel index (n*H*W + ih0*W + iw0) and ih0, iw0.
  int pbase[T::BLD], ih0[T::BLD], iw0[T::BLD];
#pragma unroll
  for (int i = 0; i < T::BLD; ++i) {
    const int p = p0 + srow + 64 * i;
    if (p < a.P) {
      const int ow = p % a.OW, t = p / a.OW, oh = t % a.OH, n = t / a.OH;
      ih0[i] = oh * a.sH - a.pH;
      iw0[i] = ow * a.sW - a.pW;
      pbase[i] = n * H * W + ih0[i] * W + iw0[i];
    } else {
      ih0[i] = -(1 << 20);  // never in bounds
      iw0[i] = 0;
      pbase[i] = 0;
    }
  }
  // Weight rows: MODE 0 reads the chunk-major packed image (capi.cpp
  // packed_offset); this thread's rows are oc0 + srow + 64*i, so oc%64 == srow.
  const int taps = a.kH * a.kW, n_ot = a.OCp / 64;
  const int wsw = (sch ^ ((srow >> 2) & 3)) * 16;
  const int8_t* wrow = a.w + (size_t)(oc0 + srow) * K + sch * 16;  // MODE 1 (stem) layout

  v4i ra[T::ALD], rb[T::BLD];
  auto gload = [&](int ks) {
    if constexpr (MODE == 0) {
      const int cpt = C / BK;  // K steps per tap
      const int tap = ks / cpt, ch = ks - tap * cpt, cb = ch * BK;
#pragma unroll
      for (int i = 0; i < T::ALD; ++i)
        ra[i] = *(const v4i*)(a.w + (((size_t)ch * n_ot + oc0 / 64 + i) * 64 + srow) * (taps * 64) +
                              tap * 64 + wsw);
      const int kh = tap / a.kW, kw = tap - kh * a.kW;
#pragma unroll
      for (int i = 0; i < T::BLD; ++i) {
        const int ih = ih0[i] + kh, iw = iw0[i] + kw;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          rb[i] = *(const v4i*)(a.x + (size_t)(pbase[i] + kh * W + kw) * C + cb + sch * 16);
        else
          rb[i] = v4i{0, 0, 0, 0};
      }
    } else {
#pragma unroll
      for (int i = 0; i < T::ALD; ++i) ra[i] = *(const v4i*)(wrow + (size_t)(64 * i) * K + ks * BK);
      const int kh = 2 * ks + (sch >> 1), kw0 = (sch & 1) * 4;
#pragma unroll
      for (int i = 0; i < T::BLD; ++i) {
        const int ih = ih0[i] + kh;
        const bool rowok = (unsigned)ih < (unsigned)H;
        const int* src = (const int*)a.x + (pbase[i] + kh * W + kw0);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int iw = iw0[i] + kw0 + t;
          rb[i][t] = (rowok && (unsigned)iw < (unsigned)W) ? src[t] : 0;
        }
      }
    }
  };
  auto lstore = [&](int buf) {
    int8_t* A = lds + buf * T::BUF;
    int8_t* B = A + TOC * BK;
#pragma unroll
    for (int i = 0; i < T::ALD; ++i) {
      const int row = srow + 64 * i;
      *(v4i*)(A + row * BK + swz(row, sch) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::BLD; ++i) {
      const int row = srow + 64 * i;
      *(v4i*)(B + row * BK + swz(row, sch) * 16) = rb[i];
    }
  };

  using Acc = typename std::conditional<F8, v16f, v16i>::type;
  Acc acc[T::FM][T::FN];
#pragma unroll
  for (int fm = 0; fm < T::FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < T::FN; ++fn) acc[fm][fn] = Acc{0};

  const int lr = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    const int8_t* A = lds + buf * T::BUF;
    const int8_t* B = A + TOC * BK;
    if constexpr (F8) {
      v4i af[2][T::FM], bf[2][T::FN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = 2 * kk + lh;
#pragma unroll
        for (int fm = 0; fm < T::FM; ++fm) {
          const int row = wo * T::WTOC + fm * 32 + lr;
          af[kk][fm] = *(const v4i*)(A + row * BK + swz(row, ch) * 16);
        }
#pragma unroll
        for (int fn = 0; fn < T::FN; ++fn) {
          const int row = wp * T::WTP + fn * 32 + lr;
          bf[kk][fn] = *(const v4i*)(B + row * BK + swz(row, ch) * 16);
        }
      }
#pragma unroll
      for (int fm = 0; fm < T::FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < T::FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              cat8(af[0][fm], af[1][fm]), cat8(bf[0][fn], bf[1][fn]), acc[fm][fn], 0, 0, 0, 0, 0, 0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = 2 * kk + lh;
      v4i af[T::FM], bf[T::FN];
#pragma unroll
      for (int fm = 0; fm < T::FM; ++fm) {
        const int row = wo * T::WTOC + fm * 32 + lr;
        af[fm] = *(const v4i*)(A + row * BK + swz(row, ch) * 16);
      }
#pragma unroll
      for (int fn = 0; fn < T::FN; ++fn) {
        const int row = wp * T::WTP + fn * 32 + lr;
        bf[fn] = *(const v4i*)(B + row * BK + swz(row, ch) * 16);
      }
#pragma unroll
      for (int fm = 0; fm < T::FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < T::FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
  };

  // Register-staged double buffer, one barrier per K step: the next step's
  // global loads are in flight while this step's MFMAs run (T14 split).
  const int nk = K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload(ks + 1);
    compute(cur);
    if (ks + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue ----------------------------------------------------
  const int OC = a.OC;
#pragma unroll
  for (int fm = 0; fm < T::FM; ++fm) {
    const int ocb = oc0 + wo * T::WTOC + fm * 32 + 4 * lh;
#pragma unroll
    for (int fn = 0; fn < T::FN; ++fn) {
      const int pix = p0 + wp * T::WTP + fn * 32 + lr;
      if (pix >= a.P) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int oc = ocb + 8 * g;  // this lane's 4 consecutive channels oc..oc+3
        if (oc >= OC) continue;
        const size_t o = (size_t)pix * OC + oc;
        if constexpr (OUT == 2) {  // raw accumulators: int32, or fp32 for F8
          using E = typename std::conditional<F8, float, int>::type;
          E* yp = (E*)a.y + o;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (oc + j < OC) yp[j] = acc[fm][fn][4 * g + j];
        } else {
          const float4 al = *(const float4*)(a.alpha + oc);
          const float4 be = *(const float4*)(a.beta + oc);
          const float alv[4] = {al.x, al.y, al.z, al.w};
          const float bev[4] = {be.x, be.y, be.z, be.w};
          float y[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) y[j] = __builtin_fmaf((float)acc[fm][fn][4 * g + j], alv[j], bev[j]);
          if constexpr (F8) {
            if constexpr (RES) {
              const int rq = *(const int*)(a.res + o);
              y[0] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8(rq, 0), a.s_res, y[0]);
              y[1] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8(rq, 1), a.s_res, y[1]);
              y[2] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8(rq, 2), a.s_res, y[2]);
              y[3] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8(rq, 3), a.s_res, y[3]);
            }
            *(unsigned*)((int8_t*)a.y + o) = enc4_f8(y[0], y[1], y[2], y[3], a.relu ? 0.f : -448.f);
          } else if constexpr (OUT == 1) {
            float* yp = (float*)a.y + o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float v = y[j];
              if (a.relu) v = v > 0.f ? v : 0.f;
              if (oc + j < OC) yp[j] = v;
            }
          } else {
            int rq = 0;
            if constexpr (RES) rq = *(const int*)(a.res + o);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if constexpr (RES) y[j] = __builtin_fmaf((float)(int)(signed char)(rq >> (8 * j)), a.s_res, y[j]);
            *(unsigned*)((int8_t*)a.y + o) = quant4(y[0], y[1], y[2], y[3], a.relu ? 0.f : -127.f);
          }
        }
      }
    }
  }
}

template <int TOC, int TP, int WOC, int MODE>
hipError_t launch_cfg(const ConvArgs& a, hipStream_t s) {
  const int ntile = (a.OCp / TOC) * ((a.P + TP - 1) / TP);
  const dim3 grid(ntile), block(NT);
  if (a.out_kind == 2) {
    hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 2, false>), grid, block, 0, s, a);
  } else if (a.out_kind == 1) {
    if constexpr (MODE == 0) hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 1, false>), grid, block, 0, s, a);
    else return hipErrorInvalidValue;
  } else if (a.res) {
    if constexpr (MODE == 0) hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 0, true>), grid, block, 0, s, a);
    else return hipErrorInvalidValue;
  } else {
    hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 0, false>), grid, block, 0, s, a);
  }
  return hipGetLastError();
}

// fp8 convs: the generic tiles only (generic packed layout, MODE 0 / stem).
template <int TOC, int TP, int WOC, int MODE>
hipError_t launch_cfg_f8(const ConvArgs& a, hipStream_t s) {
  const int ntile = (a.OCp / TOC) * ((a.P + TP - 1) / TP);
  const dim3 grid(ntile), block(NT);
  if (a.out_kind == 2) {
    hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 2, false, true>), grid, block, 0, s, a);
  } else if (a.res) {
    if constexpr (MODE == 0) hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 0, true, true>), grid, block, 0, s, a);
    else return hipErrorInvalidValue;
  } else {
    hipLaunchKernelGGL((conv_s8_kernel<TOC, TP, WOC, MODE, 0, false, true>), grid, block, 0, s, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// HBM-bound passes
// ---------------------------------------------------------------------------

// fp32 NCHW [N][3][H][W] -> int8 NHWC4: one thread = 4 consecutive pixels of a
// row: three 16-B plane loads, one 16-B store.
__global__ __launch_bounds__(256) void quantize_rgb_nhwc4_kernel(const float* __restrict__ x, int N,
                                                                 int H, int W, float inv_s,
                                                                 int8_t* __restrict__ y) {
  const int W4 = W >> 2;
  const long total = (long)N * H * W4;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int w4 = (int)(t % W4);
    const long nh = t / W4;
    const int h = (int)(nh % H), n = (int)(nh / H);
    const size_t plane = (size_t)H * W;
    const float* src = x + (size_t)n * 3 * plane + (size_t)h * W + 4 * w4;
    const float4 r = *(const float4*)(src);
    const float4 g = *(const float4*)(src + plane);
    const float4 b = *(const float4*)(src + 2 * plane);
    const float rv[4] = {r.x, r.y, r.z, r.w}, gv[4] = {g.x, g.y, g.z, g.w},
                bv[4] = {b.x, b.y, b.z, b.w};
    v4i out;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      out[j] = (sat_rne(rv[j] * inv_s) & 0xff) | ((sat_rne(gv[j] * inv_s) & 0xff) << 8) |
               ((sat_rne(bv[j] * inv_s) & 0xff) << 16);
    *(v4i*)(y + ((size_t)(n * H + h) * W + 4 * w4) * 4) = out;
  }
}

// Generic fp32 NCHW -> int8 NHWC (Cout >= C, padding channels zero).
__global__ __launch_bounds__(256) void quantize_nchw_nhwc_kernel(const float* __restrict__ x, int N,
                                                                 int C, int H, int W, int Cout,
                                                                 float inv_s,
                                                                 int8_t* __restrict__ y) {
  const long total = (long)N * H * W * Cout;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int c = (int)(t % Cout);
    const long pix = t / Cout;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H), n = (int)(nh / H);
    int q = 0;
    if (c < C) q = sat_rne(x[(((size_t)n * C + c) * H + h) * W + w] * inv_s);
    y[t] = (int8_t)q;
  }
}

__global__ __launch_bounds__(256) void quantize_rows_kernel(const float* __restrict__ x, int rows,
                                                            int cols, int ldy, float inv_s,
                                                            int8_t* __restrict__ y) {
  const int l4 = ldy >> 2;
  const long total = (long)rows * l4;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int r = (int)(t / l4), j0 = 4 * (int)(t % l4);
    unsigned packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j0 + j;
      const int q = col < cols ? sat_rne(x[(size_t)r * cols + col] * inv_s) : 0;
      packed |= ((unsigned)q & 0xffu) << (8 * j);
    }
    *(unsigned*)(y + (size_t)r * ldy + j0) = packed;
  }
}

// 3x3/s2/p1 max over int8 NHWC; one thread = 16 channels of one output pixel.
__global__ __launch_bounds__(256) void maxpool_nhwc_s8_kernel(const int8_t* __restrict__ x, int N,
                                                              int C, int H, int W, int OH, int OW,
                                                              int8_t* __restrict__ y) {
  const int cc = C >> 4;
  const long total = (long)N * OH * OW * cc;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(t % cc);
    const long pix = t / cc;
    const int ow = (int)(pix % OW);
    const long r = pix / OW;
    const int oh = (int)(r % OH), n = (int)(r / OH);
    v16c m = (v16c)(signed char)-128;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const v16c v = *(const v16c*)(x + ((size_t)(n * H + ih) * W + iw) * C + ch * 16);
        m = __builtin_elementwise_max(m, v);
      }
    }
    *(v16c*)(y + (size_t)pix * C + ch * 16) = m;
  }
}

// GAP: one thread = 4 channels of one image; exact int32 sums, then requant.
__global__ __launch_bounds__(256) void gap_nhwc_s8_kernel(const int8_t* __restrict__ x, int N, int C,
                                                          int HW, float k,
                                                          int8_t* __restrict__ y) {
  const int c4 = C >> 2;
  const long total = (long)N * c4;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % c4), n = (int)(t / c4);
    const int8_t* src = x + (size_t)n * HW * C + 4 * cg;
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < HW; ++i) {
      const int d = *(const int*)(src + (size_t)i * C);
      s0 += (signed char)(d);
      s1 += (signed char)(d >> 8);
      s2 += (signed char)(d >> 16);
      s3 += (signed char)(d >> 24);
    }
    const unsigned packed = ((unsigned)sat_rne((float)s0 * k) & 0xffu) |
                            (((unsigned)sat_rne((float)s1 * k) & 0xffu) << 8) |
                            (((unsigned)sat_rne((float)s2 * k) & 0xffu) << 16) |
                            (((unsigned)sat_rne((float)s3 * k) & 0xffu) << 24);
    *(unsigned*)(y + (size_t)n * C + 4 * cg) = packed;
  }
}

// Reference-order im2col (kernels/im2col.cu:37-54), batch honoured:
// col[n][r][oh*OW+ow], r = c*kH*kW + kh*kW + kw.
__global__ __launch_bounds__(256) void im2col_nchw_s8_kernel(const int8_t* __restrict__ x, int N,
                                                             int C, int H, int W, int kH, int kW,
                                                             int sH, int sW, int pH, int pW,
                                                             int OH, int OW,
                                                             int8_t* __restrict__ col) {
  const long cs = (long)OH * OW, K = (long)C * kH * kW;
  const long total = N * K * cs;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const long p = t % cs, nr = t / cs;
    const int r = (int)(nr % K), n = (int)(nr / K);
    const int oh = (int)(p / OW), ow = (int)(p % OW);
    const int c = r / (kH * kW), rr = r % (kH * kW), kh = rr / kW, kw = rr % kW;
    const int ih = oh * sH - pH + kh, iw = ow * sW - pW + kw;
    int8_t v = 0;
    if (ih >= 0 && iw >= 0 && ih < H && iw < W) v = x[(((size_t)n * C + c) * H + ih) * W + iw];
    col[t] = v;
  }
}

inline int grid_for(long total, int per_block = 256) {
  long g = (total + per_block - 1) / per_block;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

bool is_stem(int C, int kH, int kW) { return C == kStemC && kH == 7 && kW == 7; }

hipError_t launch_conv(const ConvArgs& a, hipStream_t s) {
  if (conv3x3s1_supported(a)) return launch_conv3x3s1(a, s);
  if (is_stem(a.C, a.kH, a.kW)) return launch_cfg<64, 256, 1, 1>(a, s);
  if (a.OCp == 64) return launch_cfg<64, 256, 1, 0>(a, s);
  return launch_cfg<128, 128, 2, 0>(a, s);
}

hipError_t launch_conv_f8(const ConvArgs& a, hipStream_t s) {
  if (is_stem(a.C, a.kH, a.kW)) return launch_cfg_f8<64, 256, 1, 1>(a, s);
  if (a.OCp == 64) return launch_cfg_f8<64, 256, 1, 0>(a, s);
  return launch_cfg_f8<128, 128, 2, 0>(a, s);
}

hipError_t launch_quantize_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cout,
                                        float inv_s, int8_t* y, hipStream_t s) {
  if (C == 3 && Cout == 4 && W % 4 == 0) {
    const long total = (long)N * H * (W / 4);
    hipLaunchKernelGGL(quantize_rgb_nhwc4_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, N, H,
                       W, inv_s, y);
  } else {
    const long total = (long)N * H * W * Cout;
    hipLaunchKernelGGL(quantize_nchw_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, N, C,
                       H, W, Cout, inv_s, y);
  }
  return hipGetLastError();
}

hipError_t launch_quantize_rows(const float* x, int rows, int cols, int ldy, float inv_s,
                                int8_t* y, hipStream_t s) {
  const long total = (long)rows * (ldy / 4);
  hipLaunchKernelGGL(quantize_rows_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, rows, cols,
                     ldy, inv_s, y);
  return hipGetLastError();
}

hipError_t launch_maxpool(const int8_t* x, int N, int C, int H, int W, int8_t* y, hipStream_t s) {
  const int OH = out_dim(H, 3, 2, 1), OW = out_dim(W, 3, 2, 1);
  const long total = (long)N * OH * OW * (C / 16);
  hipLaunchKernelGGL(maxpool_nhwc_s8_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, N, C, H, W,
                     OH, OW, y);
  return hipGetLastError();
}

// launch_gap (C % 16 == 0) lives in head.hip; this is the any-C fallback.
hipError_t launch_gap4(const int8_t* x, int N, int C, int HW, float k, int8_t* y, hipStream_t s) {
  const long total = (long)N * (C / 4);
  hipLaunchKernelGGL(gap_nhwc_s8_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, N, C, HW, k,
                     y);
  return hipGetLastError();
}

hipError_t launch_im2col_nchw(const int8_t* x, int N, int C, int H, int W, int kH, int kW, int sH,
                              int sW, int pH, int pW, int8_t* col, hipStream_t s) {
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  const long total = (long)N * C * kH * kW * OH * OW;
  hipLaunchKernelGGL(im2col_nchw_s8_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, N, C, H, W,
                     kH, kW, sH, sW, pH, pW, OH, OW, col);
  return hipGetLastError();
}

}  // namespace dlq
