// conv3x3w.hip -- stride-1 3x3 int8 conv for the wide layers (C == OC in
// {128, 256, 512} at 28x28 / 14x14 / 7x7: the nine layer2..layer4 launches
// that keep the resolution).
//
// Replaces im2col_nchw + sgemm_tiled + bn/add/relu (RK/kernels/im2col.cu:5-58,
// sgemm_tiled.cu:5-46; launched from RK/runtime/infer_e2e.cu:102-136,156-203)
// for these shapes.  The GEMM is D[oc][px] = W[oc][(tap, c)] . X[px][(tap, c)]
// with the im2col formed in LDS from a once-loaded input patch.
//
// Work item = 128 output channels x 256 consecutive output pixels; one
// 8-wave workgroup per CU walks its items (XCD-aware order: items that share
// input rows or weights run on the same XCD at the same time).  A stage is one
// 32-channel slice of the item's K: the weight block [128 oc][9 taps x 32 B]
// (pitch 304: conflict-free ds_read_b128) plus the input patch of that slice
// (32-byte pixel rows, halves swizzled by bit 3 of the patch pixel index).
// Stages stream through a 3-slot LDS-DMA ring, two stages in flight while one
// is multiplied; every wave issues the same number of LDS-DMA pieces per
// stage so the waits are exact vmcnt counts, not drains.  Each wave owns
// 64 oc x 64 px (2x2 v_mfma_i32_32x32x32_i8 tiles: one LDS read per MFMA).
//
// Epilogue without LDS: dequant*BN + residual + ReLU + requant on the MFMA
// layout, then two v_permlane32_swap per 32x32 tile turn "4 oc x 4 groups per
// lane" into 16 contiguous output channels per lane -> one 16-byte store per
// lane and tile; the residual is loaded in that store layout one stage early
// and swapped back the same way.
#include <type_traits>

#include "device_common.h"

namespace dlq {
namespace {

__device__ __attribute__((aligned(64))) int8_t g_trash_w[1024];  // sink for stores past the last pixel

// Cycle stamps for tools/probe/conv3x3w_stamps.hip (compiled out of the library).
#ifdef DLQ_STAMPS
__device__ unsigned long long g_stamps[256 * 8 * 64];
#define DLQ_STAMP(i)                                                                          \
  do {                                                                                        \
    if ((threadIdx.x & 63) == 0 && (i) < 64)                                                  \
      g_stamps[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define DLQ_STAMP(i) \
  do {               \
  } while (0)
#endif

constexpr int WTM = 128;                  // oc per item
constexpr int WTN = 256;                  // px per item
constexpr int WFM = 2;                    // 32-oc MFMA tiles per wave
constexpr int WFN = 2;                    // 32-px MFMA tiles per wave
constexpr int WMW = WTM / (32 * WFM);     // waves along oc
constexpr int WNW = WMW * (WTN / (32 * WFN));  // waves: 2 per SIMD, wave tile 64 oc x 64 px
// (a 4-wave 128 oc x 64 px tiling halves nothing that matters: one wave per
//  SIMD cannot overlap LDS latency with MFMAs; measured 1.4x slower)
constexpr int WLW = WNW;                  // of which issue the LDS-DMA (waves 0..WLW-1)
constexpr int WSC = 32;                   // input channels per stage
constexpr int WPITCH = 9 * WSC + 16;      // weight row pitch (304 = 19 x 16 B: odd -> conflict-free)
constexpr int WSTAGE_W = WTM * WPITCH;    // 38,912 B = 38 LDS-DMA pieces
constexpr int WRING = 3;

template <int W>
struct WPatch {
  static constexpr int H = W;
  static constexpr int ROWS = (WTN + W - 1) / W + 1;
  static constexpr int IMGS = (WTN + H * W - 1) / (H * W) + 1;
  static constexpr int SLOTS = ROWS + 2 * IMGS;
  static constexpr int UNITS = SLOTS * W * 2;  // 16-byte units (two per 32-channel pixel row)
  static constexpr int PIECES = (UNITS + 63) / 64;
  static constexpr int PBYTES = PIECES * 1024;
};


// OUT: 0 = int8 (fused epilogue), 2 = int32 accumulators.  XB: timing
// experiments for tools/probe (0 in the library): 1 no MFMA, 2 patch pieces
// read contiguous KiBs, 4 weight pieces all from stage block 0, 8 no epilogue,
// 16 no LDS-DMA.
template <int W, int C, int OUT, bool RES, int XB = 0>
__global__ __launch_bounds__(WNW * 64, 1) void conv3x3w_kernel(ConvArgs a) {
  using G = WPatch<W>;
  constexpr int H = W, NS = C / WSC;
  // 256 zero bytes at the end of every ring slot: a tap outside the image
  // reads the zero unit on the banks its patch address would have used, so
  // zero reads never collide with the real reads of their lane group.
  constexpr int ZREL = WSTAGE_W + G::PBYTES;
  constexpr int STAGE = ZREL + 256;
  constexpr int WP = WSTAGE_W / 1024, NPIECE = WP + G::PIECES;
  constexpr int DPW = (NPIECE + WLW - 1) / WLW;  // LDS-DMA instructions per loader wave per stage
  static_assert(DPW <= 18, "at most two DMA pieces per tap");
  constexpr int LOADS = (OUT == 0 && RES) ? WFM * WFN : 0;  // epilogue residual loads per wave
  constexpr int STORES = OUT == 0 ? WFM * WFN : 4 * WFM * WFN;  // epilogue stores per wave
  constexpr int OFF_AB = WRING * STAGE;
  constexpr int LDS_TOTAL = OFF_AB + 2 * C * 4;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  static_assert(NS >= 4, "the wait accounting assumes >= 4 stages per item");
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm = wave % WMW, wn = wave / WMW;  // wave's oc group and px group in the item
  const bool loader = wave < WLW;
  const int n_ot = a.OCp / WTM;
  const int NI = n_ot * ((a.P + WTN - 1) / WTN);
  const int Gd = gridDim.x, b = xcd_remap(blockIdx.x, Gd);
  const int nst = ((NI - b + Gd - 1) / Gd) * NS;

  DLQ_STAMP(0);
  if constexpr (OUT == 0) {
    for (int i = tid; i < a.OCp; i += WNW * 64) {
      ((float*)(lds + OFF_AB))[i] = a.alpha[i];
      ((float*)(lds + OFF_AB))[C + i] = a.beta[i];
    }
  }
  if (tid < 192) ((int*)(lds + (tid >> 6) * STAGE + ZREL))[tid & 63] = 0;
  const unsigned lds32 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int8_t*)lds;  // LDS byte address
  __syncthreads();  // before any LDS-DMA is in flight

  auto item_of = [&](int li, int& ot, int& p0) {
    const int it = b + li * Gd;
    ot = it % n_ot;
    p0 = (it / n_ot) * WTN;
  };

  // ---- issue side: this wave's DMA pieces pc = wave + 8k (wave-uniform:
  // weight piece if pc < WP, else patch piece).  Per lane a 32-bit source
  // offset for slice j = 0 (-1: outside the image -> reads x[0..15], never
  // used); slice j adds j*WSTAGE_W (weights) or j*32 (patch).  Pieces past
  // the stage's last re-issue earlier ones (same bytes, same place), and
  // stages past the end re-issue the last one into the free ring slot, so
  // every wave issues DPW pieces per stage and every wait below is a
  // compile-time count.
  int doff[DPW];
  int iss_li = -1;
  auto piece_of = [&](int k) {
    int pc = wave + k * WLW;
    return pc >= NPIECE ? pc - NPIECE : pc;
  };
  auto prep_issue = [&](int li) {
    int ot, p0;
    item_of(li, ot, p0);
    const PatchTile t = patch_tile(p0, min(p0 + WTN, a.P), W, H);
    const int units = t.slots * W * 2;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int pc = piece_of(k);
      if (pc < WP) {
        doff[k] = ot * NS * WSTAGE_W + pc * 1024 + lane * 16;
      } else {
        const int u = (pc - WP) * 64 + lane, q = u >> 1;
        const int half = (u & 1) ^ ((q >> 3) & 1);
        const int slot = q / W, col = q - slot * W;
        int n, ih;
        patch_slot(t, slot, H, n, ih);
        const bool ok = u < units && (unsigned)ih < (unsigned)H;
        doff[k] = ok ? ((n * H + ih) * W + col) * C + half * 16 : -1;
      }
    }
  };
  auto issue_piece = [&](int s, int k) {
    const int sc = s < nst ? s : nst - 1;
    const int j = sc % NS;
    const int pc = piece_of(k);
    const int8_t* src = pc < WP ? a.w + (size_t)(doff[k] + j * WSTAGE_W)
                                : a.x + (doff[k] < 0 ? (size_t)0 : (size_t)(doff[k] + j * WSC));
    if constexpr (XB & 2) {
      if (pc >= WP) src = a.x + (size_t)((sc * NPIECE + pc) % 4096) * 1024 + lane * 16;
    }
    if constexpr (XB & 4) {
      if (pc < WP) src = a.w + pc * 1024 + lane * 16;
    }
    if constexpr (!(XB & 16)) glds16_asm(src, lds32 + (s % WRING) * STAGE + pc * 1024);
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
  int a_off[WFM];  // weight fragment: row wm*32*WFM + fm*32 + lr, half lh (+ tap*32)
#pragma unroll
  for (int fm = 0; fm < WFM; ++fm) a_off[fm] = (wm * 32 * WFM + fm * 32 + lr) * WPITCH + lh * 16;
  int rel_b[WFN][9];  // patch fragment offset within a slot per (pixel tile, tap); ZREL if outside
  v16i acc[WFM][WFN];
  v4i rq[WFM][WFN] = {};  // residual in the store layout, loaded one stage early
  int cur_ot = 0, cur_p0 = 0;

  if (loader) {
    prep_for(0);
#pragma unroll
    for (int k = 0; k < DPW; ++k) issue_piece(0, k);
    prep_for(1);
#pragma unroll
    for (int k = 0; k < DPW; ++k) issue_piece(1, k);
  }

  DLQ_STAMP(1);
  for (int s = 0; s < nst; ++s) {
    const int li = s / NS, j = s - li * NS;
    DLQ_STAMP(2 + 3 * s);
    // Stage s's pieces have landed once only the younger VM ops remain:
    // stage s+1's pieces, the epilogue stores of s-1 / s-2 (an item ended
    // there) and the residual loads issued at s-1 (s ends an item).
    if (loader) {
      if ((j == 0 && s >= 1) || (j == 1 && s >= 2))
        wait_vm_const<DPW + STORES>();
      else if (j == NS - 1)
        wait_vm_const<DPW + LOADS>();
      else
        wait_vm_const<DPW>();
    } else {
      if ((j == 0 && s >= 1) || (j == 1 && s >= 2))
        wait_vm_const<STORES>();
      else if (j == NS - 1)
        wait_vm_const<LOADS>();
      else
        wait_vm_const<0>();
    }
    __builtin_amdgcn_s_barrier();
    DLQ_STAMP(3 + 3 * s);

    if (j == 0) {  // new item: fragment offsets, zero accumulators
      item_of(li, cur_ot, cur_p0);
      const PatchTile cur = patch_tile(cur_p0, min(cur_p0 + WTN, a.P), W, H);
#pragma unroll
      for (int fn = 0; fn < WFN; ++fn) {
        int base;
        unsigned m;
        patch_pixel(cur, cur_p0 + wn * 32 * WFN + fn * 32 + lr, W, H, base, m);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int q = base + (tap / 3) * W + (tap % 3) - 1;
          const int unit = 2 * q + (lh ^ ((q >> 3) & 1));  // 16-byte unit of the swizzled patch
          rel_b[fn][tap] = ((m >> tap) & 1) ? WSTAGE_W + unit * 16 : ZREL + (unit & 15) * 16;
        }
      }
#pragma unroll
      for (int fm = 0; fm < WFM; ++fm)
#pragma unroll
        for (int fn = 0; fn < WFN; ++fn) acc[fm][fn] = v16i{0};
    }
    // Residual of the item that ends at stage s+1, before stage s+2's DMA.
    if constexpr (LOADS > 0) {
      if (j == NS - 2) {
        int ot, p0;
        item_of(li, ot, p0);
#pragma unroll
        for (int fm = 0; fm < WFM; ++fm)
#pragma unroll
          for (int fn = 0; fn < WFN; ++fn) {
            const int p = p0 + wn * 32 * WFN + fn * 32 + lr;
            const size_t off = p < a.P ? (size_t)p * a.OC + ot * WTM + wm * 32 * WFM + fm * 32 + lh * 16 : 0;
            rq[fm][fn] = gload16_untracked(a.res + off);
          }
      }
    }
    if (loader) prep_for(s + 2);

    // 9 taps x one 32-deep k-step.  Fragments are read two taps ahead; stage
    // s+2's DMA pieces go out one per tap between the MFMAs.
    const int sbase = (s % WRING) * STAGE;
    constexpr int PD = (XB & 64) ? 3 : 2;  // prefetch distance in taps
    v4i fa[PD + 1][WFM], fb[PD + 1][WFN];
    auto load_tap = [&](int tap, int buf) {
#pragma unroll
      for (int fm = 0; fm < WFM; ++fm) fa[buf][fm] = *(const v4i*)(lds + sbase + a_off[fm] + tap * 32);
#pragma unroll
      for (int fn = 0; fn < WFN; ++fn) fb[buf][fn] = *(const v4i*)(lds + sbase + rel_b[fn][tap]);
    };
    // DMA pieces of stage s+2 per tap (loader waves): pieces [t*DPW/9, (t+1)*DPW/9)
    auto run_taps = [&](auto mfma_on, auto ld) {
      constexpr bool LD = decltype(ld)::value;
#pragma unroll
      for (int t = 0; t < PD; ++t) load_tap(t, t);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int k0 = tap * DPW / 9, k1 = (tap + 1) * DPW / 9;
        if (tap + PD < 9) load_tap(tap + PD, (tap + PD) % (PD + 1));
        if constexpr (LD) {
#pragma unroll
          for (int k = k0; k < k1; ++k) issue_piece(s + 2, k);
        }
        const int bu = tap % (PD + 1);
        if constexpr (decltype(mfma_on)::value) {
          if constexpr ((XB & 32) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int fm = 0; fm < WFM; ++fm)
#pragma unroll
            for (int fn = 0; fn < WFN; ++fn)
              acc[fm][fn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu][fm], fb[bu][fn], acc[fm][fn], 0, 0, 0);
          if constexpr ((XB & 32) != 0) __builtin_amdgcn_s_setprio(0);
        } else {
#pragma unroll
          for (int fm = 0; fm < WFM; ++fm) asm volatile("" ::"v"(fa[bu][fm]));
#pragma unroll
          for (int fn = 0; fn < WFN; ++fn) asm volatile("" ::"v"(fb[bu][fn]));
        }
        // interleave: the next fragments' ds_reads and this tap's DMA pieces between the MFMAs
        const int nv = LD ? k1 - k0 : 0;
        constexpr int NR = WFM + WFN, NM = WFM * WFN;
        if (tap + PD < 9) {
#pragma unroll
          for (int i = 0; i < NM; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            if (i == 2 && nv > 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
            if (i == 5 && nv > 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            if (i == 7 && nv > 2) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          }
        } else {
          if (nv > 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          if (nv > 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          if (nv > 2) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
      }
    };
    using MF = std::integral_constant<bool, !(XB & 1)>;
    if (loader)
      run_taps(MF{}, std::true_type{});
    else
      run_taps(MF{}, std::false_type{});

    DLQ_STAMP(4 + 3 * s);
    if (j != NS - 1 || (XB & 8)) continue;
    // ---- fused epilogue of the item ----
    if constexpr (OUT == 2) {
#pragma unroll
      for (int fn = 0; fn < WFN; ++fn) {
        const int p = cur_p0 + wn * 32 * WFN + fn * 32 + lr;
        const bool keep = p < a.P;
#pragma unroll
        for (int fm = 0; fm < WFM; ++fm)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int oc = cur_ot * WTM + wm * 32 * WFM + fm * 32 + 8 * g + 4 * lh;
            v4i* dst = keep ? (v4i*)((int*)a.y + (size_t)p * a.OC + oc) : (v4i*)(g_trash_w + lane * 16);
            *dst = v4i{acc[fm][fn][4 * g], acc[fm][fn][4 * g + 1], acc[fm][fn][4 * g + 2], acc[fm][fn][4 * g + 3]};
          }
      }
    } else {
      if constexpr (RES) {
        // issued at stage s-1 before the pieces of stages s+1 and s+2
        static_assert(WFM == 2 && WFN == 2, "the residual wait below names 4 registers");
        if (loader)
          asm volatile("s_waitcnt vmcnt(%4)"
                       : "+v"(rq[0][0]), "+v"(rq[0][1]), "+v"(rq[1][0]), "+v"(rq[1][1])
                       : "n"(2 * DPW)
                       : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)"
                       : "+v"(rq[0][0]), "+v"(rq[0][1]), "+v"(rq[1][0]), "+v"(rq[1][1])
                       :
                       : "memory");
      }
      const float lo = a.relu ? 0.f : -127.f;
#pragma unroll
      for (int fm = 0; fm < WFM; ++fm) {
        // alpha/beta of this lane's 16 channels (MFMA layout), read as ints
        float al[4][4], be[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = cur_ot * WTM + wm * 32 * WFM + fm * 32 + 8 * g + 4 * lh;
          const v4i a4 = *(const v4i*)(lds + OFF_AB + oc * 4);
          const v4i b4 = *(const v4i*)(lds + OFF_AB + (C + oc) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            al[g][e] = __int_as_float(a4[e]);
            be[g][e] = __int_as_float(b4[e]);
          }
        }
#pragma unroll
        for (int fn = 0; fn < WFN; ++fn) {
          unsigned r[4] = {0, 0, 0, 0};
          if constexpr (RES) {
            // store layout -> MFMA layout: (r0,r1) and (r2,r3) swaps give g = 0,2 and 1,3
            r[0] = (unsigned)rq[fm][fn][0];
            r[1] = (unsigned)rq[fm][fn][1];
            r[2] = (unsigned)rq[fm][fn][2];
            r[3] = (unsigned)rq[fm][fn][3];
            swap32(r[0], r[1]);
            swap32(r[2], r[3]);
          }
          const unsigned rg[4] = {r[0], r[2], r[1], r[3]};  // residual bytes of group g
          unsigned q[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = __builtin_fmaf((float)acc[fm][fn][4 * g + e], al[g][e], be[g][e]);
              if constexpr (RES) v[e] = __builtin_fmaf((float)(int)(signed char)(rg[g] >> (8 * e)), a.s_res, v[e]);
            }
            q[g] = quant4(v[0], v[1], v[2], v[3], lo);
          }
          // MFMA layout -> 16 contiguous channels per lane
          swap32(q[0], q[2]);
          swap32(q[1], q[3]);
          const int p = cur_p0 + wn * 32 * WFN + fn * 32 + lr;
          const bool keep = p < a.P;
          v4i* dst = keep ? (v4i*)((int8_t*)a.y + (size_t)p * a.OC + cur_ot * WTM + wm * 32 * WFM + fm * 32 + lh * 16)
                          : (v4i*)(g_trash_w + lane * 16);
          *dst = v4i{(int)q[0], (int)q[2], (int)q[1], (int)q[3]};
        }
      }
    }
  }
  DLQ_STAMP(63);
  wait_vm0();
}

int num_cus_w() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int W, int C>
hipError_t launch_wc(const ConvArgs& a, hipStream_t s) {
  const int NI = (a.OCp / WTM) * ((a.P + WTN - 1) / WTN), ncu = num_cus_w();
  const dim3 grid(NI < ncu ? NI : ncu), block(WNW * 64);
  if (a.out_kind == 2)
    hipLaunchKernelGGL((conv3x3w_kernel<W, C, 2, false>), grid, block, 0, s, a);
  else if (a.res)
    hipLaunchKernelGGL((conv3x3w_kernel<W, C, 0, true>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3w_kernel<W, C, 0, false>), grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace

bool conv3x3w_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  if (!(kH == 3 && kW == 3 && sH == 1 && sW == 1 && pH == 1 && pW == 1 && H == W && OC == C)) return false;
  return (W == 28 && C == 128) || (W == 14 && C == 256) || (W == 7 && C == 512);
}

size_t conv3x3w_packed_bytes(int OC, int C) { return (size_t)packed_oc(OC) * (C / WSC) * WPITCH; }

// OIHW q[OC][IC][3][3] -> [OCp/128][C/32][128 oc][9 taps x 32 channels + 16 pad]
void conv3x3w_pack(const int8_t* q, int OC, int IC, int C, int8_t* out) {
  const size_t total = conv3x3w_packed_bytes(OC, C);
  for (size_t i = 0; i < total; ++i) out[i] = 0;
  const int NS = C / WSC;
  for (int o = 0; o < OC; ++o)
    for (int c = 0; c < IC; ++c)
      for (int t = 0; t < 9; ++t) {
        const int ot = o / WTM, ol = o % WTM, j = c / WSC, cc = c % WSC;
        out[(((size_t)ot * NS + j) * WTM + ol) * WPITCH + t * WSC + cc] = q[((size_t)o * IC + c) * 9 + t];
      }
}

hipError_t launch_conv3x3w(const ConvArgs& a, hipStream_t s) {
  switch (a.W) {
    case 28: return launch_wc<28, 128>(a, s);
    case 14: return launch_wc<14, 256>(a, s);
    case 7: return launch_wc<7, 512>(a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dlq
