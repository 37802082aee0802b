// conv3x3s2i.hip -- stride-2 3x3 int8 conv (layer2.0 / layer3.0 / layer4.0
// conv1: C -> 2C channels, resolution halved) with the block's 1x1/s2
// downsample fused in, work items sized so that a B=256 launch is exactly
// four, two or one items per CU.
//
// Replaces, per downsampling BasicBlock (RK = CUDA/resnet18-kernel-lab/cpp/fp32):
// conv2d_nchw_im2col_gemm for conv1 + bn_launch + relu_forward
// (RK/runtime/infer_e2e.cu:161-176) AND the downsample branch's conv2d + bn
// (:187-196).  The 1x1/s2 downsample reads exactly conv1's centre tap
// (kh = kw = 1), so its MFMA takes the B fragment conv1's tap 4 already holds.
//
// Work item = 128 output channels x 196 output pixels (7 output rows of 28,
// one 14x14 image, or four 7x7 images: whole rows) -> 1024 / 512 / 256 items
// at B = 256 (no tail round on 256 CUs), 7 MFMA pixel tiles (224 >= 196).
// Waves: oc tile w & 3, pixel tiles [0,4) / [4,7) by w >> 2 (the SIMD pair
// (w, w+4) owns all 7 of one oc tile); per tile a conv and a downsample
// accumulator.
//
// LDS patch per 32-channel slice: each chunk's input rows 2*r0-1 .. 2*r1+1,
// every row stored de-interleaved (even columns, then odd: kw = 1 reads
// E[ow], kw = 2 O[ow], kw = 0 O[ow-1]) as two 16-channel planes, so all taps
// of a pixel are one base register + immediate offsets and consecutive pixels
// read consecutive 16-byte units; ow = 0's kw = 0 taps read a zero region on
// the same banks.  Stage = conv1 weights [128][9 x 32 + 16] + downsample
// weights [128][32 + 16] + patch; 2-slot LDS-DMA ring, the next stage issued
// between the MFMAs right after the barrier that opens a stage.  Epilogues as
// in conv3x3w.hip (permlane32 swaps into 16-byte stores).
//
// F8: e4m3 operands (the fp8 path), the same staged bytes and
// LDS layout: each v_mfma_f32_32x32x64_f8f6f4 takes two taps of the 32-channel
// slice (tap 8 paired with zeros, 5 MFMAs per slice); the downsample's MFMA
// takes the pair (tap 4, tap 5) with its A fragment's upper half zero, so only
// the centre tap contributes.  B pairs stream through a 3-deep register ring.
#include <type_traits>

#include "device_common.h"

namespace dlq {
namespace {

__device__ __attribute__((aligned(64))) int8_t g_trash_s2i[1024];
__device__ __attribute__((aligned(64))) int8_t g_zero_s2i[1024];  // zero halo source (+ j * 32 per slice)

// Cycle stamps for tools/probe/conv3x3s2i_probe.hip -DDLQ_STAMPS (compiled out of the library).
#ifdef DLQ_STAMPS
__device__ unsigned long long g_stamps_j[1024 * 8 * 64];
#define JSTAMP(i)                                                                                  \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && (i) < 64)                                                       \
      g_stamps_j[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define JSTAMP(i) \
  do {            \
  } while (0)
#endif

constexpr int JL = 196;               // output pixels per item
constexpr int JSC = 32;               // input channels per stage
constexpr int JWP = 9 * JSC + 16;     // conv1 weight row pitch (304 B)
constexpr int JDP = JSC + 16;         // downsample weight row pitch (48 B)
constexpr int JNW = 8;                // waves
constexpr int JOT = 128;              // output channels per item

// NSR > 0: resident weights (RW) -- all NSR stages' weight blocks are loaded
// into LDS once per workgroup and only the patch streams through the ring.
// Used when every item has the same output-channel tile (OCp == JOT: layer2.0,
// whose 1024 items would otherwise re-stream the same 88 KB four times per CU).
template <int OW, bool DS, int NSR = 0>
struct JGeo {
  static constexpr int OH = OW, WI = 2 * OW, HI = 2 * OH;  // output / input geometry
  static constexpr int RPI = OW < 14 ? OW : (OW == 14 ? 14 : 7);  // output rows per chunk
  static constexpr int IPI = JL / (RPI * OW);                 // chunks (images) per item
  static constexpr int IRC = 2 * RPI + 1;                     // input rows per chunk
  // chunk pitch in units: one spare unit for the four 7x7 images of OW = 7 so
  // that no bank quad serves more than 14 of an item's pixels (PixPerm)
  static constexpr int CS = IRC * WI + (OW == 7 ? 1 : 0);
  static constexpr int UP = (IPI * CS + 15) / 16 * 16;        // units per 16-channel plane
  static constexpr int PP = (2 * UP + 63) / 64;               // patch DMA pieces
  static constexpr int WB = JOT * JWP;                        // 38,912 = 38 pieces
  static constexpr int DB = JOT * JDP;                        // 6,144 = 6 pieces
  static constexpr int WP = (WB + (DS ? DB : 0)) / 1024;   // weight pieces (no downsample block without DS)
  static constexpr int WPC = NSR ? 0 : WP;                    // weight pieces per ring stage
  static constexpr int NPIECE = WPC + PP;
  static constexpr int W_ALL = NSR * WP * 1024;               // resident weights (stage j at j * WP KiB)
  static constexpr int OFF_P = NSR ? W_ALL : WB + DB;         // slot 0's patch
  static constexpr int ZU = 2 * WI + 16;                      // zero units (kh rows x bank spread)
  static constexpr int OFF_Z = OFF_P + PP * 1024;
  static constexpr int ZB = (ZU * 16 + 255) / 256 * 256;
  static constexpr int SLOT = NSR ? PP * 1024 + ZB : OFF_Z + ZB;  // ring slot stride
  static constexpr int OFF_AB = NSR ? W_ALL + 2 * SLOT : 2 * SLOT;  // conv alpha/beta, then ds alpha/beta
  static_assert(IPI * RPI * OW == JL, "item = whole output rows");
  static_assert((WB + DB) % 1024 == 0, "weight blocks = whole DMA pieces");
  static_assert((2 * WI + OW) * 16 < 65536, "tap offsets fit the ds_read immediate");
};

// Pixel -> lane assignment.  A B-fragment ds_read_b128 is served in 16-lane
// groups ({0-3,12-15,20-27} and {4-11,16-19,28-31} of each lane half), and a
// group is conflict-free only if its 16 pixels' tap units fall in 16
// distinct bank quads (unit mod 16).  In row order the stride-2 patch rows
// (2 input rows of 2*OW units per output row of OW pixels) shift that
// residue at every row end: 33-42 % of these launches' LDS cycles were bank
// conflicts (SQ_LDS_BANK_CONFLICT).  The D tile's pixel set is free, so the
// item's 196 pixels are dealt to the 7 tiles x 2 groups by residue: the k-th
// pixel of residue q goes to group k, lane slot q (every residue occurs <= 14
// times); the 28 spare lanes re-read a donor pixel of the missing residue and
// are flagged (0x4000) so the epilogue drops them.  Every tap adds the same
// unit offset to all lanes, so all taps stay conflict-free.
struct PixPerm {
  short px[7 * 32];
};

template <int OW>
constexpr PixPerm make_perm() {
  using G = JGeo<OW, true>;
  constexpr int LA[16] = {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27};
  constexpr int LB[16] = {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31};
  PixPerm t{};
  int cnt[16] = {}, donor[16] = {};
  for (int q = 0; q < 16; ++q) donor[q] = -1;
  for (int i = 0; i < 7 * 32; ++i) t.px[i] = -1;
  for (int p = 0; p < JL; ++p) {
    const int c = p / (G::RPI * OW), rem = p - c * (G::RPI * OW), r = rem / OW, ow = rem - r * OW;
    const int q = (c * G::CS + 2 * r * G::WI + ow) & 15;
    const int k = cnt[q]++;  // group k: tile k / 2, lane half-group k % 2
    if (donor[q] < 0) donor[q] = p;
    t.px[(k / 2) * 32 + ((k & 1) ? LB[q] : LA[q])] = (short)p;
  }
  for (int tile = 0; tile < 7; ++tile)
    for (int q = 0; q < 16; ++q) {
      if (t.px[tile * 32 + LA[q]] < 0) t.px[tile * 32 + LA[q]] = (short)(donor[q] | 0x4000);
      if (t.px[tile * 32 + LB[q]] < 0) t.px[tile * 32 + LB[q]] = (short)(donor[q] | 0x4000);
    }
  return t;
}

__constant__ PixPerm g_perm28 = make_perm<28>();
__constant__ PixPerm g_perm14 = make_perm<14>();
__constant__ PixPerm g_perm7 = make_perm<7>();

template <int OW>
__device__ __forceinline__ int perm_at(int slot) {
  if constexpr (OW == 28)
    return g_perm28.px[slot];
  else if constexpr (OW == 14)
    return g_perm14.px[slot];
  else
    return g_perm7.px[slot];
}

// RELU (int8, OUT == 0): conv1's clamp is [0, 127], requantised in the
// v_cvt_pk_u8_f32 form (device_common.h quant4_relu); the downsample keeps
// the signed clamp.
// One body per tile count (NF), shared by the four waves of a pair class:
// the DMA plan's slot kinds are the same for every wave (see below), so no
// per-wave instantiation is needed (eight of them thrashed the instruction
// cache, profiles/r05_icache2.txt).
template <int OW, int C, int OUT, bool DS, int NF, bool F8, bool RW, bool RELU = false>
__device__ __forceinline__ void s2i_body(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds,
                                         int8_t* y_ds, int8_t* lds, int wave, int mt, int f0) {
  using G = JGeo<OW, DS, RW ? C / JSC : 0>;
  constexpr int NS = C / JSC, OC = 2 * C;
  // issue slots per wave per stage: patch slots k < KPP (piece wv + 8 k),
  // then weight slots (weight piece wv + 8 (k - KPP): the conv block, then
  // the downsample block); a wave with no piece at a slot issues it masked
  constexpr int KPP = (G::PP + JNW - 1) / JNW;
  constexpr int KPW = (G::WPC + JNW - 1) / JNW;
  constexpr int DPW = KPP + KPW;
  // an empty slot (index past the count) is issued masked, with another
  // wave's piece (index - count): identical bytes to their own LDS address
  // even if the mask were ignored
  static_assert(G::PP >= JNW && (G::WPC == 0 || G::WPC >= JNW), "an empty slot duplicates piece (index - count)");
  static_assert(DPW <= 18, "at most two DMA pieces per tap");
  constexpr int STORES = OUT == 0 ? (DS ? 2 * NF : NF) : 4 * NF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int n_ot = a.OCp / JOT;
  const int NI = n_ot * ((a.P + JL - 1) / JL);
  int it0, nit;
  xcd_chunk(NI, it0, nit);
  const int nst = nit * NS;
  const unsigned lds32 = lds_addr32(lds);

  auto item_of = [&](int li, int& ot, int& p0) {
    const int it = xcd_item(it0, li);
    ot = it % n_ot;
    p0 = (it / n_ot) * JL;
  };

  // ---- DMA plan (as in conv3x3i.hip): PP patch pieces (per-lane sources,
  // halo units from a zero block) and WPC weight pieces (conv block, then
  // downsample block: a wave-uniform base + 16 * lane, the saddr form)
  constexpr int KP = KPP;
  constexpr int WCP = G::WB / 1024;            // conv weight pieces (then ds pieces)
  const int wv = wave;
  const int8_t* pptr[KP > 0 ? KP : 1];
  const int8_t* wb_c = a.w;   // the issuing item's conv / downsample weight blocks (wave-uniform)
  const int8_t* wb_d = w_ds;
  int iss_li = -1;
  auto prep_issue = [&](int li) {
    int ot, p0;
    item_of(li, ot, p0);
    wb_c = a.w + (size_t)ot * NS * G::WB;
    if constexpr (DS) wb_d = w_ds + (size_t)ot * NS * G::DB;
    const int R0 = p0 / OW;  // first global output row
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int pc0 = wv + k * JNW, pc = pc0 < G::PP ? pc0 : pc0 - G::PP;  // empty slot: another wave's piece
      const int u = pc * 64 + lane;
      const int plane = u >= G::UP ? 1 : 0, q = u - plane * G::UP;
      const int c = q / G::CS, rem = q - c * G::CS;
      const int r = rem / G::WI, pos = rem - r * G::WI;
      const int iw = pos < OW ? 2 * pos : 2 * (pos - OW) + 1;  // de-interleaved: even cols, then odd
      const int gr = R0 + c * G::RPI;  // chunk's first global output row
      const int n = gr / G::OH, ih = 2 * (gr - n * G::OH) - 1 + r;
      const bool ok = u < 2 * G::UP && c < G::IPI && r < G::IRC && n < a.N && (unsigned)ih < (unsigned)G::HI;
      // zero units: a 1 KiB zero block (slice j adds j * 32 and stays inside it)
      pptr[k] = ok ? a.x + (size_t)(((n * G::HI + ih) * G::WI + iw) * C + plane * 16) : g_zero_s2i + (lane & 3) * 16;
    }
  };
  auto issue_piece = [&](int s, int k) {  // s < nst; k < DPW (compile-time in every caller)
    const int j = s % NS;
    const unsigned slot = lds32 + (s & 1) * G::SLOT;
    if (k < KPP) {
      const int pc0 = wv + k * JNW, pc = pc0 < G::PP ? pc0 : pc0 - G::PP;
      glds16_asm_m(pptr[k < KP ? k : 0] + j * JSC, slot + G::OFF_P + pc * 1024, pc0 < G::PP);
    } else {
      const int wp0 = wv + (k - KPP) * JNW, wp = wp0 < G::WPC ? wp0 : wp0 - G::WPC;
      // the conv block, or the downsample block (a wave-uniform select, no branch)
      const int8_t* wb = wp < WCP ? wb_c + (size_t)j * G::WB : wb_d + (size_t)j * G::DB - WCP * 1024;
      glds16_saddr_m(wb + wp * 1024, (unsigned)lane * 16, slot + wp * 1024, wp0 < G::WPC);
    }
  };
  auto prep_for = [&](int s) {
    const int li = s / NS;
    if (li != iss_li) {
      prep_issue(li);
      iss_li = li;
    }
  };

  // ---- compute side: per px tile the slot-0 offsets of its kw = 1 (E[ow])
  // and kw = 0 (O[ow-1] or the zero region) taps at kh = 0; kw = 2 (O[ow]) is
  // kw = 1 + OW units, kh adds kh rows: immediate offsets.
  const int a_row = (mt * 32 + lr) * JWP + lh * 16;
  const int d_row = G::WB + (mt * 32 + lr) * JDP + lh * 16;
  int mid_off[NF], left_off[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int lp = perm_at<OW>((f0 + f) * 32 + lr) & 0x3fff;
    const int c = lp / (G::RPI * OW), rem = lp - c * (G::RPI * OW);
    const int r = rem / OW, ow = rem - r * OW;
    const int bu = c * G::CS + 2 * r * G::WI + ow;  // E[ow] of input row 2r-1
    mid_off[f] = G::OFF_P + lh * G::UP * 16 + bu * 16;
    left_off[f] = ow == 0 ? G::OFF_Z + ((bu + OW - 1) & 15) * 16 : mid_off[f] + (OW - 1) * 16;
  }
  using Acc = typename std::conditional<F8, v16f, v16i>::type;
  Acc acc[NF], accd[DS ? NF : 1];
  int cur_ot = 0, cur_p0 = 0;

  auto init = [&]() {  // LDS constants after the first DMA issue: their load latency overlaps it
    const int t = threadIdx.x;
    if constexpr (OUT == 0) {
      float* ab = (float*)(lds + G::OFF_AB);
      for (int i = t; i < a.OCp; i += JNW * 64) {
        ab[i] = a.alpha[i];
        ab[OC + i] = a.beta[i];
        if constexpr (DS) {
          ab[2 * OC + i] = al_ds[i];
          ab[3 * OC + i] = be_ds[i];
        }
      }
    }
    for (int i = t; i < G::ZU * 4; i += JNW * 64) {
      ((int*)(lds + G::OFF_Z))[i] = 0;
      ((int*)(lds + G::SLOT + G::OFF_Z))[i] = 0;
    }
  };
  if constexpr (RW) {  // every stage's weight block (one output-channel tile), once
    constexpr int NW = NS * G::WP;
    for (int pc = wave; pc < NW; pc += JNW) {
      const int j = pc / G::WP, q = pc - j * G::WP;
      const int8_t* src = q < G::WB / 1024 ? a.w + (size_t)j * G::WB + q * 1024 + lane * 16
                                           : w_ds + (size_t)j * G::DB + (q - G::WB / 1024) * 1024 + lane * 16;
      glds16_asm(src, lds32 + pc * 1024);
    }
  }
  JSTAMP(0);
  prep_for(0);
  JSTAMP(55);
#pragma unroll
  for (int k = 0; k < DPW; ++k) issue_piece(0, k);
  JSTAMP(56);
  init();  // published by stage 0's barrier
  JSTAMP(57);

  // one stage (s < nst); MORE: a stage follows (its DMA is issued in this
  // one).  int8: every stage but the last, and the last, as two
  // instantiations, so no DMA issue sits behind a runtime branch.
  // The epilogues of the item (ot, p0): conv1 (+ downsample), from acc / accd.
  auto item_epilogue = [&](int ot, int p0) {
    if constexpr (OUT == 2) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int e = perm_at<OW>((f0 + f) * 32 + lr), p = p0 + (e & 0x3fff);
        const bool keep = !(e & 0x4000) && p < a.P;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = ot * JOT + mt * 32 + 8 * g + 4 * lh;
          v4i* dst = keep ? (v4i*)((int*)a.y + (size_t)p * a.OC + oc) : (v4i*)(g_trash_s2i + lane * 16);
          if constexpr (F8)  // raw fp32 accumulators
            *dst = v4i{__float_as_int(acc[f][4 * g]), __float_as_int(acc[f][4 * g + 1]),
                       __float_as_int(acc[f][4 * g + 2]), __float_as_int(acc[f][4 * g + 3])};
          else
            *dst = v4i{acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
        }
      }
    } else {
      // probe builds: dbg 16 / 32 send the downsample / conv1 stores to the trash line
      auto epi = [&](const Acc* ac, int ab_off, float lo, int8_t* out, auto rc, bool no_store) {
        constexpr bool RL = decltype(rc)::value;
        float al[4][4], be[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = ot * JOT + mt * 32 + 8 * g + 4 * lh;
          const v4i a4 = *(const v4i*)(lds + G::OFF_AB + ab_off + oc * 4);
          const v4i b4 = *(const v4i*)(lds + G::OFF_AB + ab_off + (OC + oc) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            al[g][e] = __int_as_float(a4[e]);
            be[g][e] = __int_as_float(b4[e]);
          }
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          unsigned q[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if constexpr (F8) {
              const float a4[4] = {ac[f][4 * g], ac[f][4 * g + 1], ac[f][4 * g + 2], ac[f][4 * g + 3]};
              q[g] = epi4_f8(a4, al[g], be[g], lo);
            } else if constexpr (RL) {
              const int a4[4] = {ac[f][4 * g], ac[f][4 * g + 1], ac[f][4 * g + 2], ac[f][4 * g + 3]};
              q[g] = epi4_relu(a4, al[g], be[g]);
            } else {
              const int a4[4] = {ac[f][4 * g], ac[f][4 * g + 1], ac[f][4 * g + 2], ac[f][4 * g + 3]};
              q[g] = epi4(a4, al[g], be[g], lo);
            }
          }
          swap32(q[0], q[2]);
          swap32(q[1], q[3]);
          const int e = perm_at<OW>((f0 + f) * 32 + lr), p = p0 + (e & 0x3fff);
          const bool keep = !(e & 0x4000) && p < a.P && !no_store;
          v4i* dst = keep ? (v4i*)(out + (size_t)p * a.OC + ot * JOT + mt * 32 + lh * 16)
                          : (v4i*)(g_trash_s2i + lane * 16);
          if (DLQ_ABL(a, 128))  // probe builds: one contiguous KiB per wave-store (store-pattern ablation)
            dst = (v4i*)(out + ((((size_t)blockIdx.x * JNW + wave) * 64 + (size_t)(p0 / JL) * 8 + f) * 1024) %
                                   ((size_t)a.P * a.OC) + lane * 16);
          if (!DLQ_ABL(a, 64))  // probe builds: dbg 64 drops the int8 stores
            *dst = v4i{(int)q[0], (int)q[2], (int)q[1], (int)q[3]};
        }
      };
      constexpr float LO = F8 ? -448.f : -127.f;
      epi(acc, 0, a.relu ? 0.f : LO, (int8_t*)a.y, std::integral_constant<bool, RELU && !F8>{}, DLQ_ABL(a, 32));
      if constexpr (DS) {  // probe builds: dbg 8 skips the downsample's epilogue
        if (!DLQ_ABL(a, 8)) epi(accd, 2 * OC * 4, LO, y_ds, std::integral_constant<bool, false>{}, DLQ_ABL(a, 16));
      }
    }
  };

  // one stage (s < nst); MORE: a stage follows (its DMA is issued in this
  // one).  int8: every stage but the last, and the last, as two
  // instantiations, so no DMA issue sits behind a runtime branch.
  auto stage = [&](int s, auto more_c) {
    const int li = s / NS, j = s - li * NS;
    if (s == 0) JSTAMP(58);
    // Stage s has landed once every older VM op is done except the previous
    // item's epilogue stores (issued after this stage's DMA).
    if (j == 0 && s > 0)
      wait_vm_const<STORES>();
    else
      wait_vm_const<0>();
    if (s == 0) JSTAMP(59);
    __builtin_amdgcn_s_barrier();
    JSTAMP(1 + 2 * s);
    // (fp8: one instantiation with the runtime test -- two spill its registers)
    const bool more = decltype(more_c)::value && (!F8 || s + 1 < nst);
    if (more) prep_for(s + 1);
    // the launch's last stage issues no DMA of its own: pull the next
    // launch's first weight stages (engine forwards) into the idle patch slot
    if constexpr (!decltype(more_c)::value && !F8) prefetch_next(a.pf, wave, JNW, lds32 + ((s + 1) & 1) * G::SLOT + G::OFF_P);
    if (j == 0) {
      item_of(li, cur_ot, cur_p0);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[f] = Acc{0};
        if constexpr (DS) accd[f] = Acc{0};
      }
    }
    const int sb = (s & 1) * G::SLOT;
    if (s > 0) {
      const int d = (s & 1) ? G::SLOT : -G::SLOT;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        mid_off[f] += d;
        left_off[f] += d;
      }
    }
    const int wb = RW ? j * G::WP * 1024 : sb;  // this stage's weight block
    const int8_t* abase = lds + wb + a_row;
    if constexpr (F8) {
      constexpr int NPAIR = 5, NM = NPAIR * NF, D = 3;
      auto ld_half = [&](int tap, int f) -> v4i {
        const int kh = tap / 3, kw = tap % 3;
        const int base = kw == 0 ? left_off[f] : mid_off[f];
        return *(const v4i*)(lds + base + (kh * G::WI + (kw == 2 ? OW : 0)) * 16);
      };
      auto ld_a2 = [&](int pr) -> v8i {
        const v4i lo = *(const v4i*)(abase + (2 * pr) * 32);
        const v4i hi = 2 * pr + 1 < 9 ? *(const v4i*)(abase + (2 * pr + 1) * 32) : v4i{0, 0, 0, 0};
        return cat8(lo, hi);
      };
      auto ld_b2 = [&](int i) -> v8i {
        const int pr = i / NF, f = i - pr * NF;
        const v4i lo = ld_half(2 * pr, f);
        const v4i hi = 2 * pr + 1 < 9 ? ld_half(2 * pr + 1, f) : v4i{0, 0, 0, 0};
        return cat8(lo, hi);
      };
      v8i fa2[2], fbr[D], fd2;
      fa2[0] = ld_a2(0);
#pragma unroll
      for (int i = 0; i < D; ++i) fbr[i] = ld_b2(i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pr = 0; pr < NPAIR; ++pr) {
        if (pr + 1 < NPAIR) fa2[(pr + 1) & 1] = ld_a2(pr + 1);
        if constexpr (DS) {
          if (pr == 1) fd2 = cat8(*(const v4i*)(lds + wb + d_row), v4i{0, 0, 0, 0});  // used with pair (4, 5)
        }
        const int k0 = 2 * pr * DPW / 9, k1 = (2 * pr + 2 < 9 ? 2 * pr + 2 : 9) * DPW / 9;
        if (more && !DLQ_ABL(a, 2)) {
#pragma unroll
          for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const int i = pr * NF + f;
          acc[f] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa2[pr & 1], fbr[i % D], acc[f], 0, 0, 0, 0, 0, 0);
          if constexpr (DS) {
            if (pr == 2)
              accd[f] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fd2, fbr[i % D], accd[f], 0, 0, 0, 0, 0, 0);
          }
          if (i + D < NM) fbr[i % D] = ld_b2(i + D);
        }
      }
    } else {
    v4i fa[2], fb[NF], fd;
    auto ld_b = [&](int tap, int f) {
      const int kh = tap / 3, kw = tap % 3;
      const int base = kw == 0 ? left_off[f] : mid_off[f];
      fb[f] = *(const v4i*)(lds + base + (kh * G::WI + (kw == 2 ? OW : 0)) * 16);
    };
    fa[0] = *(const v4i*)abase;
#pragma unroll
    for (int f = 0; f < NF; ++f) ld_b(0, f);
    __builtin_amdgcn_sched_barrier(0);  // tap 0's fragment reads stay here (see conv3x3i.hip)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int bu = tap & 1;
      if (tap + 1 < 9) fa[bu ^ 1] = *(const v4i*)(abase + (tap + 1) * 32);
      if constexpr (DS) {
        if (tap == 3) fd = *(const v4i*)(lds + wb + d_row);  // the downsample's A fragment, used at tap 4
      }
      const int k0 = tap * DPW / 9, k1 = (tap + 1) * DPW / 9;
      if (more && !DLQ_ABL(a, 2)) {  // probe builds: timing without the DMA
#pragma unroll
        for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu], fb[f], acc[f], 0, 0, 0);
        if constexpr (DS) {
          if (tap == 4) accd[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fd, fb[f], accd[f], 0, 0, 0);
        }
        if (tap + 1 < 9) ld_b(tap + 1, f);
      }
      if (tap + 1 < 9) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          if (DS && tap == 4)
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA (conv + downsample)
          else
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (i == 0 && DS && tap == 3)
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // DS read: next A, ds A, B
          else if (i == 0)
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read: next A, B
          else
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if ((i == 1 && k1 > k0) || (i == 2 && k1 > k0 + 1))
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
        }
      } else {
        if (k1 > k0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (k1 > k0 + 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
      }
    }
    }  // int8 MFMA loop

    JSTAMP(2 + 2 * s);
    if (j != NS - 1) return;
    if (DLQ_ABL(a, 4)) return;  // probe builds: timing without the epilogues
    item_epilogue(cur_ot, cur_p0);
  };
  if constexpr (F8) {
    for (int s = 0; s < nst; ++s) stage(s, std::true_type{});
  } else {
    for (int s = 0; s + 1 < nst; ++s) stage(s, std::true_type{});
    if (nst > 0) stage(nst - 1, std::false_type{});
  }
  JSTAMP(62);
  wait_vm0();
  JSTAMP(63);
}

// OUT: 0 = int8 (fused epilogues), 2 = int32 conv1 accumulators (DS = false).
template <int OW, int C, int OUT, bool DS, bool F8, bool RW = false, bool RELU = false>
__global__ __launch_bounds__(JNW * 64, 1) void conv3x3s2i_kernel(ConvArgs a, const int8_t* w_ds, const float* al_ds,
                                                                 const float* be_ds, int8_t* y_ds) {
  using G = JGeo<OW, DS, RW ? C / JSC : 0>;
  constexpr int OC = 2 * C;
  constexpr int LDS_TOTAL = G::OFF_AB + (DS ? 4 : 2) * OC * 4;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // waves 0-3: pixel tiles [0,4) of oc tile w; waves 4-7: tiles [4,7)
  if (wave < 4)
    s2i_body<OW, C, OUT, DS, 4, F8, RW, RELU>(a, w_ds, al_ds, be_ds, y_ds, lds, wave, wave & 3, 0);
  else
    s2i_body<OW, C, OUT, DS, 3, F8, RW, RELU>(a, w_ds, al_ds, be_ds, y_ds, lds, wave, wave & 3, 4);
}

int num_cus_s2i() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int OW, int C, bool F8>
hipError_t launch_j(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds,
                    int8_t* y_ds, hipStream_t s) {
  const int NI = (a.OCp / JOT) * ((a.P + JL - 1) / JL), ncu = num_cus_s2i();
  const dim3 grid(NI < ncu ? NI : ncu), block(JNW * 64);
  if (a.out_kind == 2) {
    if (w_ds) return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 2, false, F8>), grid, block, 0, s, a, nullptr, nullptr, nullptr,
                       nullptr);
  } else if (w_ds) {
    const bool relu = !F8 && a.relu;  // conv1's clamp [0, 127]: the v_cvt_pk_u8_f32 epilogue
    if constexpr (OW == 28 && C == 64) {  // layer2.0: one output-channel tile -> resident weights
      if (a.OCp == JOT) {
        if (relu)
          hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, true, F8, true, true>), grid, block, 0, s, a, w_ds, al_ds,
                             be_ds, y_ds);
        else
          hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, true, F8, true>), grid, block, 0, s, a, w_ds, al_ds, be_ds,
                             y_ds);
        return hipGetLastError();
      }
    }
    if (relu)
      hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, true, F8, false, true>), grid, block, 0, s, a, w_ds, al_ds,
                         be_ds, y_ds);
    else
      hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, true, F8>), grid, block, 0, s, a, w_ds, al_ds, be_ds, y_ds);
  } else if (!F8 && a.relu) {
    // conv1 alone (the downsample computed by conv2, conv3x3i DSR): the
    // v_cvt_pk_u8_f32 epilogue, and layer2.0's resident weights
    if constexpr (OW == 28 && C == 64) {
      if (a.OCp == JOT) {
        hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, false, F8, true, true>), grid, block, 0, s, a, nullptr,
                           nullptr, nullptr, nullptr);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, false, F8, false, true>), grid, block, 0, s, a, nullptr, nullptr,
                       nullptr, nullptr);
  } else {
    hipLaunchKernelGGL((conv3x3s2i_kernel<OW, C, 0, false, F8>), grid, block, 0, s, a, nullptr, nullptr, nullptr,
                       nullptr);
  }
  return hipGetLastError();
}

template <bool F8>
hipError_t launch_s2i(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds, int8_t* y_ds,
                      hipStream_t s) {
  if (a.OCp != a.OC || a.OC != 2 * a.C || a.H != a.W || a.OW * 2 != a.W) return hipErrorInvalidValue;
  switch (a.W) {
    case 56: return a.C == 64 ? launch_j<28, 64, F8>(a, w_ds, al_ds, be_ds, y_ds, s) : hipErrorInvalidValue;
    case 28: return a.C == 128 ? launch_j<14, 128, F8>(a, w_ds, al_ds, be_ds, y_ds, s) : hipErrorInvalidValue;
    case 14: return a.C == 256 ? launch_j<7, 256, F8>(a, w_ds, al_ds, be_ds, y_ds, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

}  // namespace

// Weight images: conv3x3w_pack for conv1, downsample_pack for the 1x1 (wpack.cpp).
hipError_t launch_conv3x3s2i(const ConvArgs& a, const int8_t* w_ds, const float* al_ds, const float* be_ds,
                             int8_t* y_ds, hipStream_t s) {
  return launch_s2i<false>(a, w_ds, al_ds, be_ds, y_ds, s);
}

// e4m3 operands; the same weight images (conv3x3w_pack / downsample_pack of the codes).
hipError_t launch_conv3x3s2i_f8(const ConvArgs& a, const uint8_t* w_ds, const float* al_ds, const float* be_ds,
                                uint8_t* y_ds, hipStream_t s) {
  return launch_s2i<true>(a, (const int8_t*)w_ds, al_ds, be_ds, (int8_t*)y_ds, s);
}

}  // namespace dlq
