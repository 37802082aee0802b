// conv3x3i.hip -- stride-1 3x3 int8 conv for the wide layers (C == OC in
// {128, 256, 512} at 28x28 / 14x14 / 7x7: the nine layer2..layer4 launches
// that keep the resolution), work items sized so that a B=256 launch is
// exactly one or two items per CU.
//
// Replaces im2col_nchw + sgemm_tiled + bn/add/relu (RK/kernels/im2col.cu:5-58,
// sgemm_tiled.cu:5-46; launched from RK/runtime/infer_e2e.cu:102-136,156-203)
// for these shapes.  D[oc][px] = W[oc][(tap, c)] . X[px][(tap, c)], the
// im2col formed in LDS from a once-loaded input patch per 32-channel slice.
//
// Work item = OT output channels x 392 consecutive output pixels (14 rows of
// 28, one 14x14 image pair or eight 7x7 images: always whole output rows), so
// P = 256 * H * W splits into 512 / 128 / 32 pixel ranges and, with OT = 128 /
// 128 / 64, into 512 / 256 / 256 items: no tail round on 256 CUs.  392 px =
// 13 MFMA pixel tiles (6 % padding, vs 23 % for 256-px items whose count does
// not divide the CU count).
//
// LDS patch: per image chunk its rows plus a zero halo row above and below,
// each row with a zero column on both sides, stored as two 16-channel planes
// (plane = lane half of the MFMA operand).  Every tap of a pixel is then the
// pixel's base unit + a compile-time offset (kh * (W + 2) + kw): ds_read_b128
// with an immediate offset, no masks, no per-tap address arithmetic; the zero
// halo comes from a zero source in global memory via the same LDS-DMA.
//
// Waves: the item's MT = OT/32 oc tiles x 13 px tiles are split so that the
// two waves sharing a SIMD (w, w + 4) own 13 (MT = 4) or 7/6 (MT = 2) tiles
// of one or two oc tiles: every SIMD does the same number of MFMAs per
// k-step.  One A fragment + one B fragment per tile per tap.
//
// Stages (weight block [OT oc][9 taps x 32 B + 16 pad] + the patch of one
// 32-channel slice) stream through a 2-slot LDS-DMA ring: stage s+1 is issued
// right after the barrier that opens stage s, one piece per tap between the
// MFMAs.  Epilogue: MFMA-layout requantisation, two
// v_permlane32_swap per tile, one 16-byte store per lane and tile.
#include <type_traits>

#include "device_common.h"

namespace dlq {
namespace {

__device__ __attribute__((aligned(64))) int8_t g_trash_i[1024];  // sink for stores past the last pixel
__device__ __attribute__((aligned(64))) int8_t g_zero_i[1024];   // DMA source of the zero halo units (+ j * 32 per slice)

// Cycle stamps for tools/probe/conv3x3i_stamps.hip (compiled out of the library).
#ifdef DLQ_STAMPS
__device__ unsigned long long g_stamps_i[256 * 8 * 64];
#define ISTAMP(i)                                                                                  \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && (i) < 64)                                                       \
      g_stamps_i[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define ISTAMP(i) \
  do {            \
  } while (0)
#endif

constexpr int IL = 392;        // output pixels per item
constexpr int ISC = 32;        // input channels per stage
constexpr int IPITCH = 9 * ISC + 16;  // weight row pitch (304 B, odd multiple of 16: conflict-free)
constexpr int INW = 8;         // waves per workgroup

// SPS: 32-channel slices per stage.  The 7x7 launches (C = 512: sixteen
// one-slice stages of 58.5 MFMAs per SIMD) take two slices per stage, which
// halves their stage barriers and DMA waits; the 64-oc item's two-slice slot
// (74 KiB) still fits twice.  The wider items' slots would not.
template <int W, int SPS = 1>
struct IGeo {
  static constexpr int H = W;
  static constexpr int RPI = W < 14 ? W : 14;        // output rows per image chunk
  static constexpr int IPI = IL / (RPI * W);          // image chunks per item (1, 2, 8)
  static constexpr int OT = W == 7 ? 64 : 128;        // output channels per item
  static constexpr int MT = OT / 32;                  // oc tiles per item
  static constexpr int RW = W;                        // patch row pitch in units (compact rows)
  // Chunk pitch in units: >= the chunk's RPI + 2 rows and == RPI * W (mod 16),
  // so unit - pixel is the same mod 16 for every pixel of an item and a
  // ds_read_b128 lane group (16 consecutive pixels) hits 16 distinct bank
  // quads even across a chunk boundary (compact chunks: 26 % of the W = 7
  // launch's LDS cycles were bank conflicts, SQ_LDS_BANK_CONFLICT).
  static constexpr int CS0 = (RPI + 2) * RW;
  static constexpr int CS = CS0 + (((RPI * W - CS0) % 16) + 16) % 16;
  static constexpr int UP = (IPI * CS + 15) / 16 * 16;  // units per 16-channel plane
  static constexpr int PP = (2 * UP + 63) / 64;       // patch DMA pieces (1 KiB)
  static constexpr int ZU = 2 * W + 16;               // zero units read by the edge columns' side taps
  static constexpr int WB = OT * IPITCH;              // weight bytes per slice
  static constexpr int WP = WB / 1024;                // weight DMA pieces per slice
  static constexpr int ZB = (ZU * 16 + 255) / 256 * 256;
  // slot (slot-relative addresses): [SPS weight blocks][SPS x (patch, zero region)]
  static constexpr int WBS = SPS * WB;                // stage weight bytes
  static constexpr int PB = PP * 1024 + ZB;           // one slice's patch + zero region
  static constexpr int OFF_P = WBS;                   // slice sub's patch at OFF_P + sub * PB
  static constexpr int OFF_Z = OFF_P + PP * 1024;     // slice 0's zero region (slice sub: + sub * PB)
  static constexpr int PPS = SPS * PP, WPS = SPS * WP;  // DMA pieces per stage: patch, weights
  static constexpr int NPIECE = WPS + PPS;
  static constexpr int SLOT = WBS + SPS * PB;
  static constexpr int OFF_AB = 2 * SLOT;
  // slot bases live in registers (moved per stage); slice and tap offsets are ds_read immediates
  static_assert((SPS - 1) * PB + 2 * RW * 16 + 16 < 65536 && (SPS - 1) * WB + 8 * 32 < 65536, "immediate offsets");
  static_assert(IPI * RPI * W == IL, "item = whole output rows");
  static_assert(WB % 1024 == 0, "weight block = whole DMA pieces");
};

template <int W, bool F8>
constexpr int sps_of() {
  return W == 7 && !F8 ? 2 : 1;
}

// The DSR LDS regions past the ring and alpha/beta (conv3x3i_body DSR): the
// downsample's alpha / beta of the item's 128 channels (1 KiB), then the
// item's block-input pixels, NCH 16-byte chunks each, chunk c of pixel lp at
// unit lp * NCH + (c ^ swz(lp)) -- a B-fragment ds_read_b128's 16-lane group
// (16 of a tile's consecutive pixels, one chunk) then covers 16 distinct bank
// quads.
template <int W, int C>
struct DsrGeo {
  using G = IGeo<W, 1>;
  static constexpr int NCH = C / 32;                 // 16-byte chunks per block-input pixel (C/2 channels)
  static constexpr int NPD = (IL * NCH + 63) / 64;   // LDS-DMA pieces of the pixel region
  static constexpr int OFF_DAB = G::OFF_AB + 2 * C * 4;
  static constexpr int OFF_DS = OFF_DAB + 1024;
  static constexpr int LDS_END = OFF_DS + NPD * 1024;
  static __device__ __forceinline__ int swz(int lp) { return NCH == 4 ? (lp >> 2) & 3 : (lp >> 1) & 7; }
};

// The loaded residual staged in LDS (conv3x3i_body RLDS, 28x28 / 14x14): the
// item's 392 pixels x 128 channels, DMA'd during its second-last stage and
// read by the epilogue; pixel lp's 16-byte chunk c at lp * 128 + 16 (c ^
// ((lp >> 1) & 7)), so a ds_read_b128 lane group (16 pixels, one chunk) hits
// 16 distinct bank quads.
template <int W, int C>
struct ResGeo {
  using G = IGeo<W, 1>;
  static constexpr int OFF_RES = G::OFF_AB + 2 * C * 4;
  static constexpr int NPR = IL * G::OT / 1024;      // LDS-DMA pieces (49; W = 7 has no RLDS)
  static constexpr int LDS_END = OFF_RES + NPR * 1024;
};

// Wave -> (oc tile, first px tile, px tile count).  MT = 4: SIMD pair (w, w+4)
// = oc tile w&3, tiles [0,7) and [7,13).  MT = 2: oc tile w&1, tile groups
// [0,4) [4,7) [7,10) [10,13) by w>>1, so the pair (w, w+4) owns 7 or 6.
template <int MT>
__device__ __forceinline__ void wave_tiles(int wave, int& mt, int& f0, int& nf) {
  if constexpr (MT == 4) {
    mt = wave & 3;
    f0 = (wave >> 2) ? 7 : 0;
    nf = (wave >> 2) ? 6 : 7;
  } else {
    mt = wave & 1;
    const int g = wave >> 1;
    f0 = g == 0 ? 0 : 1 + 3 * g;
    nf = g == 0 ? 4 : 3;
  }
}

// NLD loader waves issue the LDS-DMA, lrank = this wave's rank among them
// (every wave: handing the DMA to the pairs' less loaded waves measured
// slower; so did alternating the pair's priority per tap, splitting the 13th
// tile between the pair by taps, and 12 waves (3 per SIMD); fully contiguous
// patch pieces -- what a channel-slice-major activation layout would give --
// measured only 2-5 % faster, and no DMA at all 10-15 %).
// F8: e4m3 operands (the fp8 path).  The staged bytes are the
// same; each v_mfma_f32_32x32x64_f8f6f4 takes TWO taps of the 32-channel slice
// (bytes 0-15 tap 2p, 16-31 tap 2p+1, tap 8 paired with zeros: 5 MFMAs per
// slice at twice the i8 MFMA's cycles, 10/9 of the int8 MFMA time), B
// fragments stream through a 3-deep register ring (the doubled fragment
// would not fit next to the fp32 accumulators otherwise).
// The kernel's LDS constants (zero region, alpha/beta): written after stage
// 0's DMA is issued so their global-load latency overlaps it; stage 0's
// barrier publishes them.
// s_waitcnt vmcnt(N) tied to the fragments it waits for (untracked loads,
// gload16_untracked): their later uses are ordered after the wait and no
// copy of an in-flight register can be made before it.
template <int N, int K>
__device__ __forceinline__ void wait_vm_tie_frags(v4i (&x)[K]) {
  static_assert(K == 1 || K == 2 || K == 4 || K == 8, "fragment counts of the DSR downsample");
  if constexpr (K == 1)
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(x[0]) : "n"(N) : "memory");
  else if constexpr (K == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(x[0]), "+v"(x[1]) : "n"(N) : "memory");
  else if constexpr (K == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                 : "n"(N)
                 : "memory");
}
template <int W, int C, int OUT, int SPS>
__device__ __forceinline__ void conv3x3i_init(const ConvArgs& a, int8_t* lds) {
  using G = IGeo<W, SPS>;
  const int tid = threadIdx.x;
  for (int i = tid; i < G::ZU * 4; i += INW * 64) {
#pragma unroll
    for (int sub = 0; sub < SPS; ++sub) {
      ((int*)(lds + G::OFF_Z + sub * G::PB))[i] = 0;
      ((int*)(lds + G::SLOT + G::OFF_Z + sub * G::PB))[i] = 0;
    }
  }
  if constexpr (OUT == 0) {
    for (int i = tid; i < a.OCp; i += INW * 64) {
      ((float*)(lds + G::OFF_AB))[i] = a.alpha[i];
      ((float*)(lds + G::OFF_AB))[C + i] = a.beta[i];
    }
  }
}

// The item stream of one workgroup and its LDS-DMA plan.  A stage's pieces
// are PPS patch pieces (per-lane sources: the item's rows; halo units read a
// zero block) and WPS weight pieces (1 KiB blocks of the packed image: a
// wave-uniform base + 16 * lane, the saddr form).  Wave wv issues patch
// pieces wv + NLD k at its issue slots k < KPP and weight pieces wv + NLD (k
// - KPP) at the slots after: the kind of every slot is a compile-time
// constant shared by all waves, so one code path serves every wave of a pair
// class (a per-wave instantiation multiplied the code eightfold and thrashed
// the instruction cache: 20k vs 1.3k SQC_ICACHE_MISSES per launch,
// profiles/r05_icache2.txt).  A wave with no piece at a slot (index past
// the stage's count) issues it with EXEC = 0 (glds16_*_m), and with the
// source and destination of another wave's piece of the same stage (index
// - count), so even an unmasked issue would only rewrite identical bytes at
// their own address.  With SPS slices per stage, patch piece pc is piece pc
// % PP of the stage's slice pc / PP, weight piece wp piece wp % WP of slice
// wp / WP.
template <int W, int C, int SPS, int NLD>
struct WideStream {
  using G = IGeo<W, SPS>;
  static constexpr int H = W, NSL = C / ISC, NS = NSL / SPS;
  static constexpr int KPP = (G::PPS + NLD - 1) / NLD;  // patch slots per wave per stage
  static constexpr int KPW = (G::WPS + NLD - 1) / NLD;  // weight slots per wave per stage
  static constexpr int DPW = KPP + KPW;                 // issue slots per wave per stage
  static_assert(G::PPS >= NLD && G::WPS >= NLD, "an empty slot duplicates piece (index - count)");
  const ConvArgs& a;
  int n_ot, it0, nit, nst, lane, wv, iss_li = -1;
  unsigned lds32;
  const int8_t* pptr[KPP];  // this wave's patch-piece sources for the issuing item's first slice
  const int8_t* wbase;      // the issuing item's weight blocks (wave-uniform)

  __device__ __forceinline__ WideStream(const ConvArgs& a_, int8_t* lds, int wave) : a(a_) {
    n_ot = a.OCp / G::OT;
    xcd_chunk(n_ot * ((a.P + IL - 1) / IL), it0, nit);
    nst = nit * NS;
    lane = threadIdx.x & 63;
    wv = wave;
    lds32 = lds_addr32(lds);
    wbase = a.w;
  }
  // item -> (oc tile, first pixel)
  __device__ __forceinline__ void item_of(int li, int& ot, int& p0) const {
    const int it = xcd_item(it0, li);
    ot = it % n_ot;
    p0 = (it / n_ot) * IL;
  }
  __device__ __forceinline__ void prep_issue(int li) {
    int ot, p0;
    item_of(li, ot, p0);
    // weight block [ot128][j][128][304]; a 64-oc item is half of one
    const int o128 = (ot * G::OT) >> 7, ohalf = (ot * G::OT) & 127;
    wbase = a.w + (size_t)(o128 * NSL * 128 + ohalf) * IPITCH;
    const int R0 = p0 / W;  // first global output row of the item
#pragma unroll
    for (int k = 0; k < KPP; ++k) {
      int pc = wv + k * NLD;
      if (pc >= G::PPS) pc -= G::PPS;  // an empty slot: another wave's piece (issued masked)
      const int sub = SPS > 1 && pc >= G::PP ? 1 : 0;
      const int u = (pc - sub * G::PP) * 64 + lane;
      const int plane = u >= G::UP ? 1 : 0, q = u - plane * G::UP;
      const int c = q / G::CS, rem = q - c * G::CS;
      const int r = rem / G::RW, iw = rem - r * G::RW;
      const int gr = R0 + c * G::RPI;  // chunk's first global output row
      const int n = gr / H, ih = gr - n * H + r - 1;
      const bool ok = u < 2 * G::UP && c < G::IPI && r < G::RPI + 2 && n < a.N && (unsigned)ih < (unsigned)H &&
                      (unsigned)iw < (unsigned)W;
      // zero units: a 1 KiB zero block (slice j adds j * 32 and stays inside it)
      pptr[k] = (ok ? a.x + (size_t)(((n * H + ih) * W + iw) * C + plane * 16) : g_zero_i + (lane & 3) * 16) +
                sub * ISC;
    }
  }
  __device__ __forceinline__ void issue(int s, int k) {  // s < nst; k < DPW (compile-time in every caller)
    const int j0 = (s % NS) * SPS;  // the stage's first slice
    const unsigned slot = lds32 + (s & 1) * G::SLOT;
    if (k < KPP) {
      const int pc0 = wv + k * NLD, pc = pc0 < G::PPS ? pc0 : pc0 - G::PPS;
      const int sub = SPS > 1 && pc >= G::PP ? 1 : 0;
      glds16_asm_m(pptr[k < KPP ? k : 0] + j0 * ISC, slot + G::OFF_P + sub * G::PB + (pc - sub * G::PP) * 1024,
                   pc0 < G::PPS);
    } else {
      const int wp0 = wv + (k - KPP) * NLD, wp = wp0 < G::WPS ? wp0 : wp0 - G::WPS;
      const int8_t* wsl = wbase + (size_t)j0 * 128 * IPITCH;  // the stage's first slice
      // slice 1's block (SPS = 2) sits 128 rows further: a wave-uniform select, no branch
      const int8_t* wb = SPS == 1 || wp < G::WP ? wsl : wsl + 128 * IPITCH - G::WP * 1024;
      glds16_saddr_m(wb + wp * 1024, (unsigned)lane * 16, slot + wp * 1024, wp0 < G::WPS);
    }
  }
  __device__ __forceinline__ void prep_for(int s) {
    const int li = s / NS;
    if (li != iss_li) {
      prep_issue(li);
      iss_li = li;
    }
  }
};

// RELU (int8, OUT == 0): the output clamp is [0, 127] and the requantisation
// takes the v_cvt_pk_u8_f32 form (device_common.h quant4_relu).
// DSR (int8, RES, RELU; 28x28 and 14x14): a downsampling block's conv2, whose
// residual is the block's 1x1/s2 downsample (infer_e2e.cu:187-199) computed
// here instead of read: in each item's second-to-last stage the item's block
// input pixels at (2 oh, 2 ow) (C/2 bytes each, 16-byte chunks XOR-swizzled
// by pixel) and the downsample's alpha / beta of the item's 128 channels come
// in by LDS-DMA beside the ring (the last stage's barrier publishes them); the
// last stage's start loads the wave's downsample weights (A fragments, C/64
// k-steps) into registers; the epilogue runs per tile the C/64 MFMAs on B
// fragments read from LDS (the next tile's while this tile requantises) and
// requantises downsample and conv together (device_common.h epi4_dsr_relu:
// bit-identical to the downsample's own int8 output added as the residual).
// The stride-2 conv1 of the block then runs without its fused downsample.
template <int W, int C, int OUT, bool RES, int NF, int NLD, bool F8 = false, bool RELU = false, bool DSR = false,
          bool GAP = false>
__device__ __forceinline__ void conv3x3i_body(const ConvArgs& a, int8_t* lds, int wave, int mt, int f0) {
  static_assert(!GAP || (W == 7 && C == 512 && OUT == 0 && !F8), "the pooled head follows the 7x7x512 conv");
  static_assert(!DSR || (OUT == 0 && RES && RELU && !F8 && W != 7), "the downsample residual: int8 ReLU, 28x28 / 14x14");
  constexpr bool RESL = RES && !DSR;  // the residual is loaded (DSR: computed)
  // ... through LDS (RLDS: 28x28 / 14x14 int8, where it fits beside the ring),
  // else into registers at the item's last k-step
  constexpr bool RLDS = RESL && !F8 && !GAP && W != 7 && OUT == 0;
  using RG = ResGeo<W, C>;
  constexpr int KD = C / 64;          // DSR: downsample k-steps (the block input has C/2 channels)
  using DG = DsrGeo<W, C>;
  constexpr int SPS = sps_of<W, F8>();
  using G = IGeo<W, SPS>;
  constexpr int NS = C / ISC / SPS;  // stages (SPS 32-channel slices each)
  constexpr int KSN = 9 * SPS;                            // k-steps (tap, slice) per stage
  constexpr int OFF_AB = G::OFF_AB;
  constexpr int DPW = WideStream<W, C, SPS, NLD>::DPW;  // issue slots per wave per stage
  static_assert(DPW <= 2 * KSN, "at most two DMA pieces per k-step");
  static_assert(!F8 || SPS == 1, "fp8: one slice per stage");
  static_assert(SPS <= 2, "the piece -> slice selects below");
  static_assert(NLD == INW, "every wave issues DMA pieces");
  constexpr bool loader = true;
  constexpr int STORES = OUT == 0 ? NF : 4 * NF;
  // B fragments two taps ahead for the waves with <= 6 tiles: the younger
  // wave of a SIMD pair runs alone at the end of every stage and, with its
  // fragments only one tap (6 MFMAs) ahead, waited on LDS latency there;
  // the 7-tile waves have no registers to spare for a second set
  constexpr bool PF2 = NF <= 6;

  const int tid = threadIdx.x, lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  WideStream<W, C, SPS, NLD> st(a, lds, wave);
  const int nst = st.nst;
  auto item_of = [&](int li, int& ot, int& p0) { st.item_of(li, ot, p0); };
  auto issue_piece = [&](int s, int k) { st.issue(s, k); };
  auto prep_for = [&](int s) { st.prep_for(s); };

  // ---- compute side
  const int a_row = (mt * 32 + lr) * IPITCH + lh * 16;  // + slot + tap*32
  // Per px tile the slot-0 byte offsets of its kw = 0 / 1 / 2 taps at kh = 0
  // (kh rows and slot 1 are immediate offsets; item-invariant).  A pixel in
  // the first / last column reads its kw = 0 / 2 taps from the slot's zero
  // region instead, at the unit with the real address's bank.
  int col_off[3][NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    int lp = (f0 + f) * 32 + lr;
    lp = lp < IL ? lp : IL - 1;
    const int c = lp / (G::RPI * W), rem = lp - c * (G::RPI * W);
    const int r = rem / W, ow = rem - r * W;
    const int bu = c * G::CS + r * G::RW + ow;  // tap (kh 0, kw 1): the pixel above
    const int mid = G::OFF_P + lh * G::UP * 16 + bu * 16;
    col_off[1][f] = mid;
    col_off[0][f] = ow == 0 ? G::OFF_Z + ((bu - 1) & 15) * 16 : mid - 16;
    col_off[2][f] = ow == W - 1 ? G::OFF_Z + ((bu + 1) & 15) * 16 : mid + 16;
  }
  using Acc = typename std::conditional<F8, v16f, v16i>::type;
  Acc acc[NF];
  v4i rq[NF];
  int cur_ot = 0, cur_p0 = 0;
  ISTAMP(0);
  if (loader) {
    prep_for(0);
#pragma unroll
    for (int k = 0; k < DPW; ++k) issue_piece(0, k);
  }
  if (DLQ_ABL(a, 256)) {  // probe builds: stage 0 landed from a cold L2, then the same pieces again (L2-hot)
    wait_vm_const<0>();
    __builtin_amdgcn_s_barrier();
    ISTAMP(60);
#pragma unroll
    for (int k = 0; k < DPW; ++k) issue_piece(0, k);
    wait_vm_const<0>();
    __builtin_amdgcn_s_barrier();
    ISTAMP(61);
  }
  conv3x3i_init<W, C, OUT, SPS>(a, lds);

  // one stage (s < nst); MORE: a stage follows (its DMA is issued in this
  // one).  Two instantiations -- every stage but the last, and the last --
  // so no DMA issue sits behind a runtime branch.
  auto stage = [&](int s, auto more_c) {
    const int li = s / NS, j = s - li * NS;
    // Stage s has landed once every older VM op is done except the previous
    // item's epilogue stores (issued after this stage's DMA).
    if (j == 0 && s > 0)
      wait_vm_const<STORES>();
    else
      wait_vm_const<0>();
    __builtin_amdgcn_s_barrier();
    ISTAMP(1 + 2 * s);
    // (fp8: one instantiation with the runtime test -- two spill its registers)
    const bool more = decltype(more_c)::value && (!F8 || s + 1 < nst);
    if (more && loader) prep_for(s + 1);
    // the launch's last stage issues no DMA of its own: pull the next
    // launch's first weight stages (engine forwards) into the idle slot
    if constexpr (!decltype(more_c)::value && !F8) prefetch_next(a.pf, wave, INW, lds_addr32(lds) + ((s + 1) & 1) * G::SLOT);

    if (j == 0) {
      item_of(li, cur_ot, cur_p0);
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f] = Acc{0};
    }
    v4i ads[DSR ? KD : 1];  // DSR: the downsample weights' A fragments (the item's last stage)
    constexpr bool DS_EARLY = KD <= 2;
    auto ds_aload = [&]() {
      const int o = cur_ot * G::OT + mt * 32 + lr;
#pragma unroll
      for (int kk = 0; kk < (DSR ? KD : 1); ++kk)
        ads[kk] = gload16_untracked(a.ds_w + ((size_t)((o >> 7) * KD + kk) * 128 + (o & 127)) * 48 + lh * 16);
    };
    if constexpr (RLDS) {
      if (j == NS - 2) {  // the item's residual, landed by the next stage's wait + barrier
        for (int pc = wave; pc < RG::NPR; pc += INW) {
          const int u = pc * 64 + lane, lp = u >> 3, c = (u & 7) ^ ((lp >> 1) & 7), p = cur_p0 + lp;
          const int8_t* src = p < a.P ? a.res + (size_t)p * a.OC + cur_ot * G::OT + c * 16 : g_zero_i + (lane & 3) * 16;
          glds16_asm(src, lds_addr32(lds) + RG::OFF_RES + pc * 1024);
        }
      }
    }
    if constexpr (DSR) {
      if (j == NS - 2) {
        // the item's block-input pixels and downsample alpha / beta (piece
        // NPD: lanes 0-31 alpha, 32-63 beta of the item's 128 channels)
        for (int pc = wave; pc <= DG::NPD; pc += INW) {
          const int8_t* src;
          unsigned dst;
          if (pc < DG::NPD) {
            const int u = pc * 64 + lane, lp = u / DG::NCH, c = (u - lp * DG::NCH) ^ DG::swz(lp), p = cur_p0 + lp;
            const int n = p / (W * W), r = p - n * (W * W), oh = r / W, ow = r - oh * W;
            src = lp < IL && p < a.P ? a.ds_x + (size_t)((n * 2 * W + 2 * oh) * 2 * W + 2 * ow) * (C / 2) + c * 16
                                     : g_zero_i + (lane & 3) * 16;
            dst = lds_addr32(lds) + DG::OFF_DS + pc * 1024;
          } else {
            const int o = cur_ot * G::OT + (lane & 31) * 4;
            src = (const int8_t*)((lane < 32 ? a.ds_alpha : a.ds_beta) + o);
            dst = lds_addr32(lds) + DG::OFF_DAB;
          }
          glds16_asm(src, dst);
        }
      }
      // the A fragments: ahead of the last stage's DMA (awaited in the
      // epilogue by a count of it) where the k-loop has the registers; the
      // 14x14 launch's four (16 VGPRs) wait for the epilogue (they spilled)
      if (j == NS - 1 && DS_EARLY) ds_aload();
    }
    const bool dma = more && loader && !DLQ_ABL(a, 2);  // compile-time true in library builds
    const int sb = (s & 1) * G::SLOT;
    const int8_t* abase = lds + sb + a_row;
    // this stage's slot: move the tap base registers by one slot (each tap
    // is then an immediate offset from them)
    if (s > 0) {
      const int d = (s & 1) ? G::SLOT : -G::SLOT;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        col_off[0][f] += d;
        col_off[1][f] += d;
        col_off[2][f] += d;
      }
    }
    if constexpr (F8) {
      constexpr int NPAIR = 5, NM = NPAIR * NF, D = 3;
      auto ld_half = [&](int tap, int f) -> v4i {
        return *(const v4i*)(lds + col_off[tap % 3][f] + (tap / 3) * G::RW * 16);
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
      v8i fa2[2], fbr[D];
      fa2[0] = ld_a2(0);
#pragma unroll
      for (int i = 0; i < D; ++i) fbr[i] = ld_b2(i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pr = 0; pr < NPAIR; ++pr) {
        if (pr + 1 < NPAIR) fa2[(pr + 1) & 1] = ld_a2(pr + 1);
        const int k0 = 2 * pr * DPW / 9, k1 = (2 * pr + 2 < 9 ? 2 * pr + 2 : 9) * DPW / 9;
        if (dma) {
#pragma unroll
          for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const int i = pr * NF + f;
          acc[f] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa2[pr & 1], fbr[i % D], acc[f], 0, 0, 0, 0, 0, 0);
          if (i + D < NM) fbr[i % D] = ld_b2(i + D);
          if constexpr (OUT == 0 && RESL) {
            if (pr == NPAIR - 1 && j == NS - 1) {
              const int p = cur_p0 + (f0 + f) * 32 + lr;
              const bool keep = (f0 + f) * 32 + lr < IL && p < a.P;
              const size_t off = keep ? (size_t)p * a.OC + cur_ot * G::OT + mt * 32 + lh * 16 : 0;
              rq[f] = gload16_untracked(a.res + off);
            }
          }
        }
      }
    } else {
    // k-step ks = (slice sub = ks / 9, tap = ks % 9) of the stage
    auto a_at = [&](int ks) -> v4i { return *(const v4i*)(abase + (ks / 9) * G::WB + (ks % 9) * 32); };
    auto b_off = [&](int ks, int f) {
      const int tap = ks % 9;
      return col_off[tap % 3][f] + (tap / 3) * G::RW * 16 + (ks / 9) * G::PB;
    };
    auto res_load = [&](int f) {  // the item's residual (store layout), awaited in the epilogue
      const int p = cur_p0 + (f0 + f) * 32 + lr;
      const bool keep = (f0 + f) * 32 + lr < IL && p < a.P;
      const size_t off = keep ? (size_t)p * a.OC + cur_ot * G::OT + mt * 32 + lh * 16 : 0;
      rq[f] = gload16_untracked(a.res + off);
    };
    if constexpr (PF2) {
    // B fragments two k-steps ahead: fb[ks & 1][f] holds k-step ks of tile f
    // and is re-loaded with ks + 2 right after the MFMA that consumed it (the
    // LDS latency then has two k-steps of the SIMD's MFMAs to hide in, enough
    // for a wave that runs alone at the end of a stage)
    v4i fa[2], fb[2][NF];
    auto ld_b = [&](int ks, int f) { fb[ks & 1][f] = *(const v4i*)(lds + b_off(ks, f)); };
    fa[0] = a_at(0);
#pragma unroll
    for (int f = 0; f < NF; ++f) ld_b(0, f);
    fa[1] = a_at(1);
#pragma unroll
    for (int f = 0; f < NF; ++f) ld_b(1, f);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      const int bu = ks & 1;
      const int k0 = ks * DPW / KSN, k1 = (ks + 1) * DPW / KSN;
      if (dma) {
#pragma unroll
        for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu], fb[bu][f], acc[f], 0, 0, 0);
        if (f == NF - 1 && ks + 2 < KSN) fa[bu] = a_at(ks + 2);
        if (ks + 2 < KSN && !DLQ_ABL(a, 8)) ld_b(ks + 2, f);  // probe builds: dbg 8 re-uses k-steps 0/1's B
        if constexpr (OUT == 0 && RESL && !RLDS) {
          if (ks == KSN - 1 && j == NS - 1) res_load(f);
        }
      }
      if (ks + 2 < KSN) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (i == NF - 1)
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read (B + the A two k-steps ahead)
          else
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read (B)
          if ((i == 1 && k1 > k0) || (i == 3 && k1 > k0 + 1))
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
        }
      } else {
        if (k1 > k0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (k1 > k0 + 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
      }
    }
    } else {
    // A double-buffered per k-step; each B fragment is re-loaded for the next
    // k-step right after the MFMA that consumed it (one register set per tile).
    v4i fa[2], fb[NF];
    auto ld_b = [&](int ks, int f) { fb[f] = *(const v4i*)(lds + b_off(ks, f)); };
    fa[0] = a_at(0);
#pragma unroll
    for (int f = 0; f < NF; ++f) ld_b(0, f);
    // keep k-step 0's fragment reads here: left to the scheduler they were sunk
    // into its MFMA slots and serialised (one lgkmcnt(0) per MFMA)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      const int bu = ks & 1;
      if (ks + 1 < KSN) fa[bu ^ 1] = a_at(ks + 1);
      const int k0 = ks * DPW / KSN, k1 = (ks + 1) * DPW / KSN;
      if (dma) {
#pragma unroll
        for (int k = k0; k < k1; ++k) issue_piece(s + 1, k);
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[f] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[bu], fb[f], acc[f], 0, 0, 0);
        if (ks + 1 < KSN && !DLQ_ABL(a, 8)) ld_b(ks + 1, f);  // probe builds: dbg 8 re-uses k-step 0's B
        if constexpr (OUT == 0 && RESL && !RLDS) {
          // into the registers this tile's last B fragment just freed
          if (ks == KSN - 1 && j == NS - 1) res_load(f);
        }
      }
      if (ks + 1 < KSN) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (i == 0)
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read (next k-step's A + this tile's B)
          else
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if ((i == 1 && k1 > k0) || (i == 3 && k1 > k0 + 1))
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
        }
      } else {
        if (k1 > k0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (k1 > k0 + 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
      }
    }
    }  // PF2
    }  // int8 MFMA loop

    ISTAMP(2 + 2 * s);
    if (j != NS - 1 || DLQ_ABL(a, 4)) return;  // probe builds: timing without the epilogue
    // GAP: the item's outputs are also staged in LDS for the pooling: in the
    // launch's last stage in the idle slot (past the prefetch pieces' first
    // KiB), no wait; in an earlier item's last stage the idle slot is
    // receiving the next item's stage 0, so this stage's slot is used, once
    // every wave is past its last fragment read (a barrier: the epilogues
    // then no longer overlap the slower waves' MFMAs)
    constexpr bool LAST_STAGE = !decltype(more_c)::value;
    const int gstage = LAST_STAGE ? (((s + 1) & 1) * G::SLOT + 1024) : sb;
    if constexpr (GAP && !LAST_STAGE) __builtin_amdgcn_s_barrier();
    static_assert(!GAP || 1024 + IL * 64 <= G::SLOT, "the pooling stage fits a slot");
    (void)gstage;
    // ---- fused epilogue of the item ----
    if constexpr (OUT == 2) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int lp = (f0 + f) * 32 + lr, p = cur_p0 + lp;
        const bool keep = lp < IL && p < a.P;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int oc = cur_ot * G::OT + mt * 32 + 8 * g + 4 * lh;
          v4i* dst = keep ? (v4i*)((int*)a.y + (size_t)p * a.OC + oc) : (v4i*)(g_trash_i + lane * 16);
          if constexpr (F8)  // raw fp32 accumulators
            *dst = v4i{__float_as_int(acc[f][4 * g]), __float_as_int(acc[f][4 * g + 1]),
                       __float_as_int(acc[f][4 * g + 2]), __float_as_int(acc[f][4 * g + 3])};
          else
            *dst = v4i{acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
        }
      }
    } else if constexpr (DSR) {
      // the A fragments, issued before this stage's DMA: younger than them
      // at most the fewest unmasked pieces any wave issued (a lower bound on
      // what vmcnt counts), none in the launch's last stage
      constexpr int YOUNG = decltype(more_c)::value && DS_EARLY ? G::PPS / NLD + G::WPS / NLD : 0;
      if constexpr (!DS_EARLY) ds_aload();
      wait_vm_tie_frags<YOUNG>(ads);
      // tile f's downsample accumulators (B fragments from the pixel region)
      auto ds_acc = [&](int f) {
        int lp = (f0 + f) * 32 + lr;
        lp = lp < IL ? lp : IL - 1;
        const int8_t* base = lds + DG::OFF_DS + lp * DG::NCH * 16;
        v16i ad = v16i{0};
#pragma unroll
        for (int kk = 0; kk < KD; ++kk)
          ad = __builtin_amdgcn_mfma_i32_32x32x32_i8(ads[kk], *(const v4i*)(base + (((2 * kk + lh) ^ DG::swz(lp)) << 4)),
                                                     ad, 0, 0, 0);
        return ad;
      };
      // 28x28: the next tile's MFMAs run beside this tile's requantisation;
      // 14x14 (four MFMAs per tile): one tile at a time (a second set spilled)
      constexpr bool PIPE = KD <= 2;
      v16i adn = PIPE ? ds_acc(0) : v16i{0};
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        // one tile per scheduling region: hoisting later tiles' fragment
        // reads above this one spilled the epilogue's registers
        __builtin_amdgcn_sched_barrier(0);
        const v16i ad = PIPE ? adn : ds_acc(f);
        if (PIPE && f + 1 < NF) adn = ds_acc(f + 1);
        unsigned q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          // alpha / beta of conv and downsample for this group's 4 channels,
          // from LDS per tile (registers are what this epilogue is short of)
          const int ol = mt * 32 + 8 * g + 4 * lh, oc = cur_ot * G::OT + ol;
          const v4i v[4] = {*(const v4i*)(lds + OFF_AB + oc * 4), *(const v4i*)(lds + OFF_AB + (C + oc) * 4),
                            *(const v4i*)(lds + DG::OFF_DAB + ol * 4), *(const v4i*)(lds + DG::OFF_DAB + 512 + ol * 4)};
          float ab[4][4];
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) ab[t][e] = __int_as_float(v[t][e]);
          const int ac[4] = {acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
          const int adc[4] = {ad[4 * g], ad[4 * g + 1], ad[4 * g + 2], ad[4 * g + 3]};
          q[g] = epi4_dsr_relu(ac, ab[0], ab[1], adc, ab[2], ab[3], a.s_res);
        }
        swap32(q[0], q[2]);
        swap32(q[1], q[3]);
        const int lp = (f0 + f) * 32 + lr, p = cur_p0 + lp;
        const bool keep = lp < IL && p < a.P;
        v4i* dst = keep ? (v4i*)((int8_t*)a.y + (size_t)p * a.OC + cur_ot * G::OT + mt * 32 + lh * 16)
                        : (v4i*)(g_trash_i + lane * 16);
        *dst = v4i{(int)q[0], (int)q[2], (int)q[1], (int)q[3]};
      }
    } else {
      const float lo = a.relu ? 0.f : (F8 ? -448.f : -127.f);
      float al[4][4], be[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int oc = cur_ot * G::OT + mt * 32 + 8 * g + 4 * lh;
        const v4i a4 = *(const v4i*)(lds + OFF_AB + oc * 4);
        const v4i b4 = *(const v4i*)(lds + OFF_AB + (C + oc) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          al[g][e] = __int_as_float(a4[e]);
          be[g][e] = __int_as_float(b4[e]);
        }
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        unsigned r[4] = {0, 0, 0, 0};
        if constexpr (RLDS) {
          int lp = (f0 + f) * 32 + lr;
          lp = lp < IL ? lp : IL - 1;
          rq[f] = *(const v4i*)(lds + RG::OFF_RES + lp * 128 + (((2 * mt + lh) ^ ((lp >> 1) & 7)) << 4));
        } else if constexpr (RES) {
          // younger than rq[f]: rq[f+1..NF-1] and the stores of tiles 0..f-1
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(rq[f]) : "n"(NF - 1) : "memory");
        }
        if constexpr (RES) {
          r[0] = (unsigned)rq[f][0];
          r[1] = (unsigned)rq[f][1];
          r[2] = (unsigned)rq[f][2];
          r[3] = (unsigned)rq[f][3];
          swap32(r[0], r[1]);
          swap32(r[2], r[3]);
        }
        const unsigned rg[4] = {r[0], r[2], r[1], r[3]};
        unsigned q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if constexpr (F8) {
            const float ac[4] = {acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
            if constexpr (RES)
              q[g] = epi4_res_f8(ac, al[g], be[g], rg[g], a.s_res, lo);
            else
              q[g] = epi4_f8(ac, al[g], be[g], lo);
          } else if constexpr (RELU) {
            const int ac[4] = {acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
            if constexpr (RES)
              q[g] = epi4_res_relu(ac, al[g], be[g], rg[g], a.s_res);
            else
              q[g] = epi4_relu(ac, al[g], be[g]);
          } else {
            const int ac[4] = {acc[f][4 * g], acc[f][4 * g + 1], acc[f][4 * g + 2], acc[f][4 * g + 3]};
            if constexpr (RES)
              q[g] = epi4_res(ac, al[g], be[g], rg[g], a.s_res, lo);
            else
              q[g] = epi4(ac, al[g], be[g], lo);
          }
        }
        swap32(q[0], q[2]);
        swap32(q[1], q[3]);
        const int lp = (f0 + f) * 32 + lr, p = cur_p0 + lp;
        const bool keep = lp < IL && p < a.P;
        v4i* dst = keep ? (v4i*)((int8_t*)a.y + (size_t)p * a.OC + cur_ot * G::OT + mt * 32 + lh * 16)
                        : (v4i*)(g_trash_i + lane * 16);
        if (DLQ_ABL(a, 128))  // probe builds: one contiguous KiB per wave-store (store-pattern ablation)
          dst = (v4i*)((int8_t*)a.y + ((((size_t)blockIdx.x * INW + wave) * 64 + (size_t)(cur_p0 / IL) * 8 + f) * 1024) %
                                          ((size_t)a.P * a.OC) + lane * 16);
        if (!DLQ_ABL(a, 64))  // probe builds: dbg 64 drops the int8 stores
          *dst = v4i{(int)q[0], (int)q[2], (int)q[1], (int)q[3]};
        if constexpr (GAP) {  // [392 px][64 ch] staging, 16-byte chunk c at c ^ (px & 3)
          if (lp < IL)
            *(v4i*)(lds + gstage + lp * 64 + 16 * ((2 * mt + lh) ^ (lp & 3))) = v4i{(int)q[0], (int)q[2], (int)q[1], (int)q[3]};
        }
      }
      if constexpr (GAP) {
        // The item's 8 whole images x 64 channels, pooled from the staged
        // bytes by all 8 waves: thread = (image, 8 channels, pixel group of
        // 8); the ReLU outputs are 0..127, so two channels add in the two
        // 16-bit halves of one int32 (49 x 127 < 2^16) -- exact integer sums
        // as gap16_kernel's; the 8 pixel groups of a row of lanes reduce by
        // three DPP row shifts into its lane 7, which requantises (sat_rne,
        // as gap16_kernel) and stores the 8 codes the FC reads
        // (infer_e2e.cu:417-425).
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes
        __builtin_amdgcn_s_barrier();
        {
          const int t = threadIdx.x, nl = t >> 6, cg8 = (t >> 3) & 7, pg = t & 7;
          const int n = cur_p0 / 49 + nl;
          unsigned sm[4] = {0u, 0u, 0u, 0u};  // channels {0,2} {1,3} {4,6} {5,7} of the group
#pragma unroll
          for (int jj = 0; jj < 7; ++jj) {
            const int i = pg + 8 * jj, px = nl * 49 + i;
            if (i < 49) {
              const v2i v = *(const v2i*)(lds + gstage + px * 64 + 16 * ((cg8 >> 1) ^ (px & 3)) + 8 * (cg8 & 1));
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                sm[2 * h] += (unsigned)v[h] & 0x00ff00ffu;
                sm[2 * h + 1] += ((unsigned)v[h] >> 8) & 0x00ff00ffu;
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {  // row_shr 1, 2, 4 (out-of-row lanes read 0): lane 7 of each 8 = the sum
            sm[i] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)sm[i], 0x111, 0xf, 0xf, true);
            sm[i] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)sm[i], 0x112, 0xf, 0xf, true);
            sm[i] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)sm[i], 0x114, 0xf, 0xf, true);
          }
          if (n < a.N && pg == 7) {
            unsigned o[2] = {0u, 0u};
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int b = 0; b < 4; ++b) {  // channel 4h + b: half b >> 1 of sm[2h + (b & 1)]
                const unsigned v = (sm[2 * h + (b & 1)] >> (16 * (b >> 1))) & 0xffffu;
                o[h] |= ((unsigned)sat_rne((float)(int)v * a.gap_k) & 0xffu) << (8 * b);
              }
            *(v2i*)(a.gap_y + (size_t)n * C + cur_ot * G::OT + cg8 * 8) = v2i{(int)o[0], (int)o[1]};
          }
        }
      }
    }
    };
  if constexpr (F8) {
    for (int s = 0; s < nst; ++s) stage(s, std::true_type{});
  } else {
    for (int s = 0; s + 1 < nst; ++s) stage(s, std::true_type{});
    if (nst > 0) stage(nst - 1, std::false_type{});
  }
  ISTAMP(62);
  wait_vm0();
  ISTAMP(63);
}

template <int W, int C, int OUT, bool RES, bool F8 = false, bool RELU = false, bool DSR = false, bool GAP = false>
__global__ __launch_bounds__(INW * 64, 1) void conv3x3i_kernel(ConvArgs a) {
  using G = IGeo<W, sps_of<W, F8>()>;
  constexpr int OFF_AB = G::OFF_AB;
  constexpr bool RLDS = RES && !DSR && !F8 && !GAP && W != 7 && OUT == 0;
  constexpr int LDS_TOTAL = DSR ? DsrGeo<W, C>::LDS_END : RLDS ? ResGeo<W, C>::LDS_END : OFF_AB + 2 * C * 4;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const int tid = threadIdx.x;
  int mt, f0, nf;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  wave_tiles<G::MT>(wave, mt, f0, nf);
  // one instantiation per tile count (the DMA plan's slot kinds are the same
  // for every wave, WideStream): two bodies per kernel
  if constexpr (G::MT == 4) {
    if (wave < 4)
      conv3x3i_body<W, C, OUT, RES, 7, INW, F8, RELU, DSR, GAP>(a, lds, wave, mt, f0);
    else
      conv3x3i_body<W, C, OUT, RES, 6, INW, F8, RELU, DSR, GAP>(a, lds, wave, mt, f0);
  } else {
    if (wave < 2)
      conv3x3i_body<W, C, OUT, RES, 4, INW, F8, RELU, DSR, GAP>(a, lds, wave, mt, f0);
    else
      conv3x3i_body<W, C, OUT, RES, 3, INW, F8, RELU, DSR, GAP>(a, lds, wave, mt, f0);
  }
  (void)nf;
}

int num_cus_i() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int W, int C, bool F8 = false>
hipError_t launch_ci(const ConvArgs& a, hipStream_t s) {
  using G = IGeo<W>;
  const int NI = (a.OCp / G::OT) * ((a.P + IL - 1) / IL), ncu = num_cus_i();
  const dim3 grid(NI < ncu ? NI : ncu), block(INW * 64);
  if (a.out_kind == 2)
    hipLaunchKernelGGL((conv3x3i_kernel<W, C, 2, false, F8>), grid, block, 0, s, a);
  else if (!F8 && a.relu && a.res)
    hipLaunchKernelGGL((conv3x3i_kernel<W, C, 0, true, F8, true>), grid, block, 0, s, a);
  else if (!F8 && a.relu)
    hipLaunchKernelGGL((conv3x3i_kernel<W, C, 0, false, F8, true>), grid, block, 0, s, a);
  else if (a.res)
    hipLaunchKernelGGL((conv3x3i_kernel<W, C, 0, true, F8>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3i_kernel<W, C, 0, false, F8>), grid, block, 0, s, a);
  return hipGetLastError();
}

template <int W, int C>
hipError_t launch_ci_dsr(const ConvArgs& a, hipStream_t s) {
  using G = IGeo<W, sps_of<W, false>()>;
  const int NI = (a.OCp / G::OT) * ((a.P + IL - 1) / IL), ncu = num_cus_i();
  const dim3 grid(NI < ncu ? NI : ncu), block(INW * 64);
  hipLaunchKernelGGL((conv3x3i_kernel<W, C, 0, true, false, true, true>), grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace

// conv2 of a downsampling block with the downsample residual computed in its
// epilogue (conv3x3i_body DSR): int8 output, ReLU, no loaded residual; the
// block input has C/2 channels at twice the resolution.
hipError_t launch_conv3x3i_dsr(const ConvArgs& a, hipStream_t s) {
  if (a.OCp != a.OC || a.C != a.OC || a.H != a.W || a.out_kind != 0 || !a.relu || a.res || !a.ds_x || !a.ds_w ||
      !a.ds_alpha || !a.ds_beta || a.ds_C * 2 != a.C)
    return hipErrorInvalidValue;
  if ((long long)a.N * (2 * a.H) * (2 * a.W) * a.ds_C >= (1LL << 31)) return hipErrorInvalidValue;
  switch (a.W) {
    case 28: return a.C == 128 ? launch_ci_dsr<28, 128>(a, s) : hipErrorInvalidValue;
    case 14: return a.C == 256 ? launch_ci_dsr<14, 256>(a, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;  // 7x7x512: the LDS holds no pixel region beside its two-slice ring
}

// e4m3 operands, same shapes and weight image layout (conv3x3w_pack of the codes).
hipError_t launch_conv3x3i_f8(const ConvArgs& a, hipStream_t s) {
  if (a.OCp != a.OC || a.C != a.OC || a.H != a.W) return hipErrorInvalidValue;
  switch (a.W) {
    case 28: return a.C == 128 ? launch_ci<28, 128, true>(a, s) : hipErrorInvalidValue;
    case 14: return a.C == 256 ? launch_ci<14, 256, true>(a, s) : hipErrorInvalidValue;
    case 7: return a.C == 512 ? launch_ci<7, 512, true>(a, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

// Weight image: conv3x3w_pack (wpack.cpp).
hipError_t launch_conv3x3i(const ConvArgs& a, hipStream_t s) {
  if (a.ds_x) return launch_conv3x3i_dsr(a, s);
  if (a.gap_y) {  // the pooled head after the last conv: 7x7x512, int8, ReLU, residual
    if (a.OCp != a.OC || a.C != 512 || a.OC != 512 || a.H != 7 || a.W != 7 || a.out_kind != 0 || !a.relu || !a.res)
      return hipErrorInvalidValue;
    using G = IGeo<7, sps_of<7, false>()>;
    const int NI = (a.OCp / G::OT) * ((a.P + IL - 1) / IL), ncu = num_cus_i();
    hipLaunchKernelGGL((conv3x3i_kernel<7, 512, 0, true, false, true, false, true>), dim3(NI < ncu ? NI : ncu),
                       dim3(INW * 64), 0, s, a);
    return hipGetLastError();
  }
  if (a.OCp != a.OC || a.C != a.OC || a.H != a.W) return hipErrorInvalidValue;
  switch (a.W) {
    case 28: return a.C == 128 ? launch_ci<28, 128>(a, s) : hipErrorInvalidValue;
    case 14: return a.C == 256 ? launch_ci<14, 256>(a, s) : hipErrorInvalidValue;
    case 7: return a.C == 512 ? launch_ci<7, 512>(a, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

}  // namespace dlq
