// stem.hip -- fused ResNet-18 stem: input quantisation + conv1 7x7/s2/p3 (+BN,
// ReLU, requant) + maxpool 3x3/s2/p1 in one persistent kernel.
//
// Replaces (RK = CUDA/resnet18-kernel-lab/cpp/fp32): the input upload
// (RK/runtime/infer_e2e.cu:255-256), conv2d_nchw_im2col_gemm for conv1
// (:259-270, im2col_nchw + sgemm_tiled), bn_launch + relu_forward (:272-280)
// and maxpool2d_3x3_s2p1_nchw (:282-293).  The conv1 output (64 x 112 x 112
// per image, 4x the pooled size) never reaches HBM.
//
// Space-to-depth: the 224x224x3 fp32 image is read as a 112x112 grid of
// 16-byte "super-pixels" [dy][dx][c] (2x2 pixels x RGB+0), quantised on the
// fly.  The 7x7/s2 conv becomes a 4x4/s1 conv over super-pixels whose taps
// cover input rows/cols 2*o-4 .. 2*o+3 (kh = 2*ky+dy-1; kh = -1 carries a zero
// weight), i.e. K = 16 taps x 16 B = 256 = 8 steps of v_mfma_i32_32x32x32_i8,
// and every B fragment is one 16-byte-aligned ds_read_b128 of consecutive
// super-pixels (conflict-free).
//
// Work item = a band of 4 pooled rows (x 56) of one image = 9 conv rows x 112
// (the 9th conv row is the pool halo shared with the band above, recomputed).
// One 512-thread workgroup per CU walks bands; the next band's fp32 input is
// loaded into registers while the current band's MFMAs run.
#include "device_common.h"

namespace dlq {
namespace {

constexpr int PR = 4;                 // pooled rows per band
constexpr int CR = 2 * PR + 1;        // conv rows per band
constexpr int SR = CR + 3;            // super-pixel rows per band
constexpr int SC = 115;               // super-pixel cols (-2 .. 112)
constexpr int CPX = CR * 112;         // conv pixels per band (1008)
constexpr int NW = 8;                 // waves
constexpr int NTH = NW * 64;
constexpr int FN = 4;                 // 32-px MFMA tiles per wave (8 waves x 4 x 32 = 1024 >= 1008)
constexpr int WPITCH = 272;           // LDS row pitch of the weight image (256 + 16: conflict-free)
constexpr int UNITS = SR * SC;        // super-pixels per band (1380)
constexpr int UPT = (UNITS + NTH - 1) / NTH;  // per thread (3)

constexpr int OFF_P = 0;                          // patch: SR x SC x 16 B
constexpr int OFF_W = OFF_P + SR * SC * 16;       // weights: 64 x 272 B
constexpr int OFF_C = OFF_W + 64 * WPITCH;        // conv tile: CR x 112 x 64 B (chunk-swizzled)
constexpr int OFF_AB = OFF_C + CPX * 64;          // alpha, beta: 64 + 64 floats
constexpr int LDS_TOTAL = OFF_AB + 512;
static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");

struct StemArgs {
  const float* x;      // [N][3][224][224]
  const int8_t* w;     // [64][256]  (oc, ky, kx, dy, dx, c)
  const float* alpha;  // [64] output-grid units
  const float* beta;   // [64]
  int8_t* y;           // [N][56][56][64]
  float inv_s;         // 1 / input scale
  int N;
  int dbg;             // ablation bits (timing builds only): 1 MFMA, 2 input loads, 4 epilogue+pool, 8 patch store
};

__global__ __launch_bounds__(NTH, 1) void stem_fused_kernel(StemArgs a) {
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int nbands = a.N * (56 / PR);

  // weights (once per workgroup) + epilogue constants
  for (int i = tid; i < 64 * 16; i += NTH) {
    const int oc = i >> 4, t = i & 15;
    *(v4i*)(lds + OFF_W + oc * WPITCH + t * 16) = *(const v4i*)(a.w + oc * 256 + t * 16);
  }
  if (tid < 64) {
    ((float*)(lds + OFF_AB))[tid] = a.alpha[tid];
    ((float*)(lds + OFF_AB))[64 + tid] = a.beta[tid];
  }

  // Prefetch registers: UPT super-pixels x (3 channels x 2 rows) float2.
  float2 pf[UPT][6];
  auto load_band = [&](int band) {
    const int n = band / (56 / PR), py0 = (band % (56 / PR)) * PR;
    const int sy0 = 2 * py0 - 1 - 2;  // super row of patch row 0 (conv row 2*py0-1, tap ky=0)
    const float* img = a.x + (size_t)n * 3 * 224 * 224;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = tid + k * NTH;
      const int sr = u / SC, sc = u - sr * SC;
      const int sy = sy0 + sr, sx = sc - 2;
      const bool ok = u < UNITS && (unsigned)sy < 112u && (unsigned)sx < 112u;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
          pf[k][c * 2 + dy] = ok && !(a.dbg & 2) ? *(const float2*)(img + ((size_t)c * 224 + 2 * sy + dy) * 224 + 2 * sx)
                                 : make_float2(0.f, 0.f);
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = tid + k * NTH;
      if (u >= UNITS) continue;
      unsigned w4[4];  // bytes [dy][dx][c], c = 3 is zero
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          unsigned v = 0;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const float f = dx ? pf[k][c * 2 + dy].y : pf[k][c * 2 + dy].x;
            v |= ((unsigned)sat_rne(f * a.inv_s) & 0xffu) << (8 * c);
          }
          w4[dy * 2 + dx] = v;
        }
      *(v4i*)(lds + OFF_P + u * 16) = v4i{(int)w4[0], (int)w4[1], (int)w4[2], (int)w4[3]};
    }
  };

  // lane-constant A offsets
  int a_off[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) a_off[fm] = OFF_W + (fm * 32 + lr) * WPITCH + lh * 16;
  // lane pixel -> patch offset of super tap (0,0)
  int b_off[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    int px = (wave * FN + fn) * 32 + lr;
    px = px < CPX ? px : CPX - 1;
    const int r = px / 112, ox = px - r * 112;
    b_off[fn] = OFF_P + (r * SC + ox) * 16;
  }

  int band = blockIdx.x;
  if (band < nbands) load_band(band);
  for (; band < nbands; band += gridDim.x) {
    __syncthreads();  // previous band's conv tile fully pooled, patch free
    if (!(a.dbg & 8)) store_patch();
    __syncthreads();
    if (band + (int)gridDim.x < nbands) load_band(band + gridDim.x);  // in flight during the MFMAs

    v16i acc[2][FN];
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = v16i{0};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (a.dbg & 1) break;
      const int t = 2 * kk + lh, ky = t >> 2, kx = t & 3;  // this lane's super tap
      v4i af[2], bf[FN];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) af[fm] = *(const v4i*)(lds + a_off[fm] + kk * 32);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) bf[fn] = *(const v4i*)(lds + b_off[fn] + (ky * SC + kx) * 16);
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }

    if (a.dbg & 4) {  // keep the accumulators live
      if (acc[0][0][0] == 0x7fffffff && acc[1][FN - 1][15] == 0x7fffffff) a.y[0] = 1;
      continue;
    }
    // epilogue: BN*requant + ReLU -> int8 conv tile [r][ox][64] (chunk-swizzled by pixel)
    const float* s_al = (const float*)(lds + OFF_AB);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int px = (wave * FN + fn) * 32 + lr;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ol = fm * 32 + 8 * g + 4 * lh;
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = __builtin_fmaf((float)acc[fm][fn][4 * g + j], s_al[ol + j], s_al[64 + ol + j]);
          const unsigned q = quant4(v[0], v[1], v[2], v[3], 0.f);
          if (px < CPX)
            *(unsigned*)(lds + OFF_C + px * 64 + (((ol >> 4) ^ ((px >> 2) & 3)) << 4) + ((ol >> 2) & 3) * 4) = q;
        }
    }
    __syncthreads();

    // 3x3/s2/p1 max pool of the band -> pooled int8 NHWC, 16 channels per lane
    const int n = band / (56 / PR), py0 = (band % (56 / PR)) * PR;
    for (int u = tid; u < PR * 56 * 4; u += NTH) {
      const int ch = u & 3, pp = u >> 2, ppy = pp / 56, ppx = pp - ppy * 56;
      v16c m = (v16c)(signed char)-128;
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int r = 2 * ppy + dr;
        if (py0 == 0 && r == 0) continue;  // conv row -1: pool padding
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          const int ox = 2 * ppx - 1 + dc;
          if (ox < 0) continue;
          const int px = r * 112 + ox;
          const v16c v = *(const v16c*)(lds + OFF_C + px * 64 + ((ch ^ ((px >> 2) & 3)) << 4));
          m = __builtin_elementwise_max(m, v);
        }
      }
      *(v16c*)(a.y + (((size_t)n * 56 + py0 + ppy) * 56 + ppx) * 64 + ch * 16) = m;
    }
  }
}

int num_cus_stem() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace

size_t stem_packed_bytes() { return 64 * 256; }

// OIHW int8 q[64][3][7][7] -> [64][ky 4][kx 4][dy 2][dx 2][c 4], kh = 2ky+dy-1.
void pack_stem_weights(const int8_t* q, int8_t* out) {
  for (int i = 0; i < 64 * 256; ++i) out[i] = 0;
  for (int o = 0; o < 64; ++o)
    for (int ky = 0; ky < 4; ++ky)
      for (int kx = 0; kx < 4; ++kx)
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx) {
            const int kh = 2 * ky + dy - 1, kw = 2 * kx + dx - 1;
            if (kh < 0 || kw < 0) continue;
            for (int c = 0; c < 3; ++c)
              out[o * 256 + (((ky * 4 + kx) * 2 + dy) * 2 + dx) * 4 + c] = q[((o * 3 + c) * 7 + kh) * 7 + kw];
          }
}

hipError_t launch_stem_fused(const float* x, int N, const int8_t* w, const float* alpha, const float* beta,
                             float inv_s, int8_t* y, hipStream_t s) {
  StemArgs a{x, w, alpha, beta, y, inv_s, N, debug_bits()};
  const int nb = N * (56 / PR), ncu = num_cus_stem();
  hipLaunchKernelGGL(stem_fused_kernel, dim3(nb < ncu ? nb : ncu), dim3(NTH), 0, s, a);
  return hipGetLastError();
}

}  // namespace dlq
