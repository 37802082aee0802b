// conv3x3s2.hip -- stride-2 3x3 int8 conv (layer2.0 / layer3.0 / layer4.0
// conv1: C -> 2C channels, resolution halved) with the block's 1x1/s2
// downsample conv fused in.
//
// Replaces, per downsampling BasicBlock (RK = CUDA/resnet18-kernel-lab/cpp/fp32):
// conv2d_nchw_im2col_gemm for conv1 + bn_launch + relu_forward
// (RK/runtime/infer_e2e.cu:161-176) AND the downsample branch's conv2d + bn
// (:187-196).  The 1x1/s2 downsample reads exactly the centre tap (kh = kw =
// 1) of conv1's im2col, so its B fragment is the one conv1 already loaded: the
// fused launch reads the block input once and writes both outputs (conv1 ->
// BN -> ReLU -> int8, and downsample -> BN -> int8 in its own scale).
//
// Work item = 128 output channels x 128 output pixels; 8 waves = 2 (64 oc) x 4
// (32 px).  A stage is one 32-channel slice: conv1 weights [128][9 taps x 32 +
// 16] (pitch 304, conflict-free), downsample weights [128][32 + 16] (pitch
// 48), and the input patch: the stride-2 tile's input rows, columns stored
// de-interleaved (even columns, then odd) so that every tap reads consecutive
// patch positions for consecutive output pixels (16-byte halves swizzled by
// bit 3 of the position, as in conv3x3w.hip).  Two-slot LDS-DMA ring (the
// stride-2 patch is twice the stride-1 one), exact vmcnt counts, epilogue
// through v_permlane32_swap into 16-byte stores.
#include <cstdlib>

#include "device_common.h"

namespace dlq {
namespace {

__device__ __attribute__((aligned(64))) int8_t g_trash_s2[1024];

constexpr int S2TM = 128;               // oc per item
constexpr int S2TN = 128;               // output px per item
constexpr int S2NW = 8;                 // waves: 2 (oc) x 4 (px)
constexpr int S2SC = 32;                // input channels per stage
constexpr int S2WP = 9 * S2SC + 16;     // conv1 weight row pitch (304 B)
constexpr int S2DP = S2SC + 16;         // downsample weight row pitch (48 B: 3 units, odd)
constexpr int S2W_BYTES = S2TM * S2WP;  // 38,912 = 38 pieces
constexpr int S2D_BYTES = S2TM * S2DP;  // 6,144 = 6 pieces

template <int OW>
struct S2Patch {
  static constexpr int OH = OW, W = 2 * OW;  // output rows/cols, input width
  static constexpr int ROWS = (S2TN + OW - 1) / OW + 1;            // output rows a tile can touch
  static constexpr int IMGS = (S2TN + OH * OW - 1) / (OH * OW) + 1;  // images a tile can touch
  static constexpr int SLOTS = 2 * ROWS + 2 * IMGS + 1;            // input rows
  static constexpr int UNITS = SLOTS * W * 2;                      // 16-byte units of 32-channel rows
  static constexpr int PIECES = (UNITS + 63) / 64;
  static constexpr int PBYTES = PIECES * 1024;
};

// The stride-2 patch of output tile [p0, pend): image n0's input rows
// 2*oh0-1 .. (cnt0 slots), then each further image's rows -1 .. (2*OH+1 per
// full image).  Input rows -1 are never loaded (their taps read zeros).
struct S2Tile {
  int n0, oh0, cnt0, slots;
};

__device__ __forceinline__ S2Tile s2_tile(int p0, int pend, int OW) {
  const int OH = OW;
  S2Tile t;
  const int R0 = p0 / OW, R1 = (pend - 1) / OW;
  t.n0 = R0 / OH;
  t.oh0 = R0 - t.n0 * OH;
  const int n1 = R1 / OH, oh1 = R1 - n1 * OH;
  t.cnt0 = (n1 == t.n0) ? 2 * (oh1 - t.oh0) + 3 : 2 * (OH - t.oh0) + 1;
  t.slots = (n1 == t.n0) ? t.cnt0 : t.cnt0 + (n1 - t.n0 - 1) * (2 * OH + 1) + 2 * oh1 + 3;
  return t;
}

__device__ __forceinline__ void s2_slot(const S2Tile& t, int slot, int OH, int& n, int& ih) {
  if (slot < t.cnt0) {
    n = t.n0;
    ih = 2 * t.oh0 - 1 + slot;
  } else {
    const int s2 = slot - t.cnt0;
    n = t.n0 + 1 + s2 / (2 * OH + 1);
    ih = s2 % (2 * OH + 1) - 1;
  }
}

// OUT: 0 = int8 (fused epilogues), 2 = int32 conv1 accumulators (DS = false).
template <int OW, int C, int OUT, bool DS>
__global__ __launch_bounds__(S2NW * 64, 1) void conv3x3s2_kernel(ConvArgs a, const int8_t* w_ds,
                                                                 const float* alpha_ds, const float* beta_ds,
                                                                 int8_t* y_ds) {
  using G = S2Patch<OW>;
  constexpr int OH = OW, W = G::W, H = 2 * OH, NS = C / S2SC;
  constexpr int OFF_DW = S2W_BYTES, OFF_P = OFF_DW + S2D_BYTES, ZREL = OFF_P + G::PBYTES;
  constexpr int STAGE = ZREL + 256;
  constexpr int WP = S2W_BYTES / 1024, DPC = S2D_BYTES / 1024;
  constexpr int NPIECE = WP + DPC + G::PIECES;
  constexpr int DPW = (NPIECE + S2NW - 1) / S2NW;  // LDS-DMA pieces per wave per stage
  constexpr int STORES = OUT == 0 ? (DS ? 4 : 2) : 8;
  constexpr int OFF_AB = 2 * STAGE;
  constexpr int OCN = 2 * C;  // output channels
  constexpr int LDS_TOTAL = OFF_AB + 4 * OCN * 4;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  static_assert(NS >= 2 && DPW <= 18, "stage accounting");
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const unsigned lds32 = lds_addr32(lds);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;  // 64-oc half, 32-px quarter of the item
  const int n_ot = a.OCp / S2TM;
  const int NI = n_ot * ((a.P + S2TN - 1) / S2TN);
  const int Gd = gridDim.x, b = xcd_remap(blockIdx.x, Gd);
  const int nst = ((NI - b + Gd - 1) / Gd) * NS;
  float* s_ab = (float*)(lds + OFF_AB);  // alpha, beta, alpha_ds, beta_ds

  if constexpr (OUT == 0) {
    for (int i = tid; i < OCN; i += S2NW * 64) {
      s_ab[i] = a.alpha[i];
      s_ab[OCN + i] = a.beta[i];
      if constexpr (DS) {
        s_ab[2 * OCN + i] = alpha_ds[i];
        s_ab[3 * OCN + i] = beta_ds[i];
      }
    }
  }
  if (tid < 128) ((int*)(lds + (tid >> 6) * STAGE + ZREL))[tid & 63] = 0;
  __syncthreads();

  auto item_of = [&](int li, int& ot, int& p0) {
    const int it = b + li * Gd;
    ot = it % n_ot;
    p0 = (it / n_ot) * S2TN;
  };

  // ---- issue side: piece pc = wave + 8k: conv1 weights (pc < WP), downsample
  // weights (< WP + DPC), patch.  32-bit offsets for slice j = 0; slice j adds
  // j*block (weights) or j*32 (patch; -1 = outside the image).
  int doff[DPW];
  int iss_li = -1;
  auto piece_of = [&](int k) {
    const int pc = wave + k * S2NW;
    return pc >= NPIECE ? pc - NPIECE : pc;
  };
  auto prep_issue = [&](int li) {
    int ot, p0;
    item_of(li, ot, p0);
    const S2Tile t = s2_tile(p0, min(p0 + S2TN, a.P), OW);
    const int units = t.slots * W * 2;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int pc = piece_of(k);
      if (pc < WP) {
        doff[k] = ot * NS * S2W_BYTES + pc * 1024 + lane * 16;
      } else if (pc < WP + DPC) {
        doff[k] = ot * NS * S2D_BYTES + (pc - WP) * 1024 + lane * 16;
      } else {
        const int u = (pc - WP - DPC) * 64 + lane, q = u >> 1;
        const int half = (u & 1) ^ ((q >> 3) & 1);
        const int slot = q / W, pos = q - slot * W;
        const int col = pos < W / 2 ? 2 * pos : 2 * (pos - W / 2) + 1;
        int n, ih;
        s2_slot(t, slot, OH, n, ih);
        const bool ok = u < units && (unsigned)ih < (unsigned)H;
        doff[k] = ok ? ((n * H + ih) * W + col) * C + half * 16 : -1;
      }
    }
  };
  auto issue_piece = [&](int s, int k) {
    const int sc = s < nst ? s : nst - 1;
    const int j = sc % NS;
    const int pc = piece_of(k);
    const int8_t* src;
    if (pc < WP)
      src = a.w + (size_t)(doff[k] + j * S2W_BYTES);
    else if (pc < WP + DPC)
      src = DS ? w_ds + (size_t)(doff[k] + j * S2D_BYTES) : a.w;
    else
      src = a.x + (doff[k] < 0 ? (size_t)0 : (size_t)(doff[k] + j * S2SC));
    glds16_asm(src, lds32 + (s & 1) * STAGE + pc * 1024);
  };
  auto prep_for = [&](int s) {
    const int sc = s < nst ? s : nst - 1;
    const int li = sc / NS;
    if (li != iss_li) {
      prep_issue(li);
      iss_li = li;
    }
  };

  // ---- compute side
  int a_off[2], d_off[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    a_off[fm] = (wm * 64 + fm * 32 + lr) * S2WP + lh * 16;
    d_off[fm] = OFF_DW + (wm * 64 + fm * 32 + lr) * S2DP + lh * 16;
  }
  int rel_b[9];  // patch fragment offset per tap within a slot (zero unit if outside the image)
  v16i acc[2], accd[2];
  int cur_ot = 0, cur_p0 = 0;

  prep_for(0);
#pragma unroll
  for (int k = 0; k < DPW; ++k) issue_piece(0, k);

  for (int s = 0; s < nst; ++s) {
    const int li = s / NS, j = s - li * NS;
    // Stage s's pieces have landed once only the epilogue stores of s-1 (if an
    // item ended there) are younger.
    if (j == 0 && s >= 1)
      wait_vm_const<STORES>();
    else
      wait_vm_const<0>();
    __builtin_amdgcn_s_barrier();

    if (j == 0) {
      item_of(li, cur_ot, cur_p0);
      const S2Tile t = s2_tile(cur_p0, min(cur_p0 + S2TN, a.P), OW);
      const int p = cur_p0 + wn * 32 + lr;
      int slot0 = 0, ow = 0, oh = 0;
      const bool live = p < a.P;
      if (live) {
        const int n = p / (OH * OW), r = p - n * (OH * OW);
        oh = r / OW;
        ow = r - oh * OW;
        slot0 = (n == t.n0) ? 2 * (oh - t.oh0) : t.cnt0 + (n - t.n0 - 1) * (2 * OH + 1) + 2 * oh;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3;
        const int pos = kw == 1 ? ow : W / 2 + ow - 1 + (kw >> 1);
        const int q = (slot0 + kh) * W + pos;
        const bool ok = live && !(kh == 0 && oh == 0) && !(kw == 0 && ow == 0);
        const int unit = 2 * q + (lh ^ ((q >> 3) & 1));
        rel_b[tap] = ok ? OFF_P + unit * 16 : ZREL + (unit & 15) * 16;
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) {
        acc[fm] = v16i{0};
        accd[fm] = v16i{0};
      }
    }
    prep_for(s + 1);

    // 9 taps (+ the downsample on the centre tap); fragments two taps ahead,
    // stage s+1's DMA pieces spread over the taps.
    const int sbase = (s & 1) * STAGE;
    v4i fa[3][2], fb[3];
    auto load_tap = [&](int tap, int buf) {
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) fa[buf][fm] = *(const v4i*)(lds + sbase + a_off[fm] + tap * 32);
      fb[buf] = *(const v4i*)(lds + sbase + rel_b[tap]);
    };
    v4i fd[2];
    load_tap(0, 0);
    load_tap(1, 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int k0 = tap * DPW / 9, k1 = (tap + 1) * DPW / 9;
      if (tap + 2 < 9) load_tap(tap + 2, (tap + 2) % 3);
      if (DS && tap == 2) {
#pragma unroll
        for (int fm = 0; fm < 2; ++fm) fd[fm] = *(const v4i*)(lds + sbase + d_off[fm]);
      }
#pragma unroll
      for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
      const int bu = tap % 3;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) acc[fm] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu][fm], fb[bu], acc[fm], 0, 0, 0);
      if (DS && tap == 4) {
#pragma unroll
        for (int fm = 0; fm < 2; ++fm) accd[fm] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fd[fm], fb[bu], accd[fm], 0, 0, 0);
      }
    }

    if (j != NS - 1) continue;
    // ---- epilogue(s) of the item
    const int p = cur_p0 + wn * 32 + lr;
    const bool keep = p < a.P;
    if constexpr (OUT == 2) {
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = cur_ot * S2TM + wm * 64 + fm * 32 + 8 * g + 4 * lh;
          v4i* dst = keep ? (v4i*)((int*)a.y + (size_t)p * a.OC + oc) : (v4i*)(g_trash_s2 + lane * 16);
          *dst = v4i{acc[fm][4 * g], acc[fm][4 * g + 1], acc[fm][4 * g + 2], acc[fm][4 * g + 3]};
        }
    } else {
      auto epi = [&](const v16i& ac, int fm, int ab, float lo, int8_t* out) {
        unsigned q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = cur_ot * S2TM + wm * 64 + fm * 32 + 8 * g + 4 * lh;
          const v4i a4 = *(const v4i*)(s_ab + ab * OCN + oc);
          const v4i b4 = *(const v4i*)(s_ab + (ab + 1) * OCN + oc);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf((float)ac[4 * g + e], __int_as_float(a4[e]), __int_as_float(b4[e]));
          q[g] = quant4(v[0], v[1], v[2], v[3], lo);
        }
        const v4i o = mfma_to_store16(q[0], q[1], q[2], q[3]);
        v4i* dst = keep ? (v4i*)(out + (size_t)p * a.OC + cur_ot * S2TM + wm * 64 + fm * 32 + lh * 16)
                        : (v4i*)(g_trash_s2 + lane * 16);
        *dst = o;
      };
      const float lo = a.relu ? 0.f : -127.f;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) epi(acc[fm], fm, 0, lo, (int8_t*)a.y);
      if constexpr (DS) {
#pragma unroll
        for (int fm = 0; fm < 2; ++fm) epi(accd[fm], fm, 2, -127.f, y_ds);
      }
    }
  }
  wait_vm0();
}

template <int OW, int C>
hipError_t launch_s2(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds, int8_t* y_ds,
                     hipStream_t s, int ncu) {
  const int NI = (a.OCp / S2TM) * ((a.P + S2TN - 1) / S2TN);
  const dim3 grid(NI < ncu ? NI : ncu), block(S2NW * 64);
  if (a.out_kind == 2)
    hipLaunchKernelGGL((conv3x3s2_kernel<OW, C, 2, false>), grid, block, 0, s, a, w_ds, al_ds, be_ds, y_ds);
  else if (w_ds)
    hipLaunchKernelGGL((conv3x3s2_kernel<OW, C, 0, true>), grid, block, 0, s, a, w_ds, al_ds, be_ds, y_ds);
  else
    hipLaunchKernelGGL((conv3x3s2_kernel<OW, C, 0, false>), grid, block, 0, s, a, w_ds, al_ds, be_ds, y_ds);
  return hipGetLastError();
}

int num_cus_s2() {
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

bool conv3x3s2_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  if (!(kH == 3 && kW == 3 && sH == 2 && sW == 2 && pH == 1 && pW == 1 && H == W && OC == 2 * C)) return false;
  return (W == 56 && C == 64) || (W == 28 && C == 128) || (W == 14 && C == 256);
}

size_t downsample_packed_bytes(int OC, int C) { return (size_t)packed_oc(OC) * (C / S2SC) * S2DP; }

// 1x1 weights q[OC][IC] -> [OCp/128][C/32][128 oc][32 channels + 16 zero]
void downsample_pack(const int8_t* q, int OC, int IC, int C, int8_t* out) {
  const size_t total = downsample_packed_bytes(OC, C);
  for (size_t i = 0; i < total; ++i) out[i] = 0;
  const int NS = C / S2SC;
  for (int o = 0; o < OC; ++o)
    for (int c = 0; c < IC; ++c) {
      const int ot = o / S2TM, ol = o % S2TM, j = c / S2SC, cc = c % S2SC;
      out[(((size_t)ot * NS + j) * S2TM + ol) * S2DP + cc] = q[(size_t)o * IC + c];
    }
}

// The 196-px item kernel (conv3x3s2i.hip) by default; DLQ_S2_128=1 keeps
// this file's 128-px item kernel (same weight images) for A/B timing.
hipError_t launch_conv3x3s2(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds,
                            int8_t* y_ds, hipStream_t s) {
  static const bool v128 = [] {
    const char* e = std::getenv("DLQ_S2_128");
    return e && e[0] == '1';
  }();
  if (!v128) return launch_conv3x3s2i(a, w_ds, al_ds, be_ds, y_ds, s);
  const int ncu = num_cus_s2();
  switch (a.W) {
    case 56: return launch_s2<28, 64>(a, w_ds, al_ds, be_ds, y_ds, s, ncu);
    case 28: return launch_s2<14, 128>(a, w_ds, al_ds, be_ds, y_ds, s, ncu);
    case 14: return launch_s2<7, 256>(a, w_ds, al_ds, be_ds, y_ds, s, ncu);
  }
  return hipErrorInvalidValue;
}

}  // namespace dlq
