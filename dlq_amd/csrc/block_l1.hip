// block_l1.hip -- one layer1 basic block of ResNet-18 (64 channels at 56x56:
// conv3x3-BN-ReLU, conv3x3-BN, + identity, ReLU) as ONE launch.
//
// Replaces, for this shape, the reference's basic_block_forward
// (RK/runtime/infer_e2e.cu:156-203: two im2col_nchw + sgemm_tiled convs,
// bn_launch, add_inplace, relu_forward) -- i.e. two conv launches of
// conv3x3.hip here.  The intermediate activation never leaves the CU, the
// block input is read from HBM once (plus an L2-hot re-read as the residual),
// and each intermediate row is computed exactly once.
//
// Work decomposition: one workgroup per image (persistent over images
// b, b+G, ...).  The images of a workgroup form one stream of "global rows"
// (image j = rows [56j, 56j+56)), walked in phases of 8 rows; in phase g
// (G = 8g):
//   conv1 waves (0-3): intermediate rows [G, G+8) from input rows [G-1, G+9)
//   conv2 waves (4-7): output rows [G-9, G-1) from intermediate rows [G-10, G)
//   all waves:         LDS-DMA of input rows [G+9, G+17) for phase g+1
// so conv2 trails conv1 by one phase and nothing waits inside a phase; one
// barrier per phase.  (block_l1_sp_kernel's last phase gives conv2 nine rows,
// so the image's last output row needs no phase of its own.)
//
// LDS layout: two rings (input, intermediate) of 18 rows + one zero row,
// each split into four channel planes (plane p = channels 16p .. 16p+15, 16 B
// per pixel).  A plane row is 64 units of 16 B: units 0 and 57 are zero
// padding (the conv's left/right zero columns), units 1..56 the pixels.  With
// 16-byte pixels, 16 consecutive pixels cover all 64 banks, so the pixel
// fragments need no swizzle, and a tap's address is its row's base plus an
// immediate offset (16*kw for the column, 2 planes for the second 32
// channels): the k-loop issues ds_read_b128 with no address arithmetic.
// Taps in rows outside the image read the zero row.
//
// Each wave owns one conv and 32 of its 64 output channels and keeps that
// weight slice (32 oc x 576 K = 72 VGPRs) and its alpha/beta in registers for
// the life of the kernel, so the only LDS operand traffic is the pixel
// fragment.  A job = 32 oc x 64 pixels x 576 K (36 v_mfma_i32_32x32x32_i8 in
// four independent accumulation chains); per phase 14 conv1 + 14 conv2 jobs,
// dealt so that each SIMD (waves w and w+4) gets exactly 7.
//
// Epilogues (bit-identical to conv3x3.hip / oracle.c): conv1 y =
// fma(acc, a1, b1) -> ReLU -> rne -> int8 written to the intermediate ring;
// conv2 y = fma(acc, a2, b2) + s_res * x -> ReLU -> rne -> int8 to HBM.
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "device_common.h"

namespace dlq {

__device__ __attribute__((aligned(64))) int8_t g_trash_b[1024];  // sink for stores of pixels past the end
__device__ __attribute__((aligned(64))) int8_t g_zero_b[64];     // DMA source of the zero padding units

namespace {

#ifdef DLQ_STAMPS
// timing-probe builds: per-wave cycle totals by section (no VM ops in the loop)
__device__ unsigned long long g_bstamps[256 * 8 * 128];
#define BT_DECL unsigned long long bt_acc[6] = {0, 0, 0, 0, 0, 0}, bt_prev = __builtin_amdgcn_s_memtime()
#define BT(k)                                              \
  do {                                                     \
    const unsigned long long bt_now = __builtin_amdgcn_s_memtime(); \
    bt_acc[k] += bt_now - bt_prev;                         \
    bt_prev = bt_now;                                      \
  } while (0)
#define BT_STORE()                                                                                 \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0)                                                                   \
      for (int q_ = 0; q_ < 6; ++q_) g_bstamps[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 128 + q_] = bt_acc[q_]; \
  } while (0)
#else
#define BT_DECL
#define BT(k) \
  do {        \
  } while (0)
#define BT_STORE() \
  do {             \
  } while (0)
#endif

#ifndef BL1_TEST
#define BL1_TEST 0  // timing probe builds only: 1/2 conv2/conv1 waves idle, 7 no residual loads, 8 no stores
#endif

constexpr int LW = 56;               // image height = width
constexpr int LC = 64;               // channels
constexpr int RPH = 8;               // rows per phase
constexpr int NR = 18;               // ring rows (slot NR = the zero row)
constexpr int PROW = 1024;           // plane row: 64 units of 16 B (pad, 56 pixels, pad, 6 unused)
constexpr int PL = (NR + 1) * PROW;  // one channel plane of a ring
constexpr int RING = 4 * PL;
constexpr int OFF_IN = 0;
constexpr int OFF_MID = RING;
constexpr int LDS_TOTAL = 2 * RING;
static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
static_assert(2 * PL + 32 < 65536, "ds_read immediate offset");
constexpr int KS = 18;  // 9 taps x two 32-channel k-steps

struct BlockArgs {
  const int8_t* x;   // block input [N][56][56][64]
  int8_t* y;         // block output, same shape
  const int8_t* w1;  // generic packed 3x3 weights (64 oc x 9 taps x 64 B, chunk-swizzled)
  const int8_t* w2;
  const float* a1;
  const float* b1;
  const float* a2;
  const float* b2;
  float s_res;  // residual scale in conv2's output-grid units
  int N;
  Prefetch pf;  // the next launch's first weight stages (engine forwards)
};

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int pos_mod(int v, int m) { return ((v % m) + m) % m; }

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ds_read_b128 (register address + immediate offset) the compiler does not
// track: completion only via wait_lgkm_tie, which also orders the register's
// later uses after the wait -- so hipcc can neither sink a prefetch next to
// its use nor collapse the fragment rotation.
template <int OFF>
__device__ __forceinline__ v4i ds_read16(unsigned addr) {
  v4i r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void wait_lgkm_tie(v4i& x, v4i& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_lgkm_tie8(v8i& x, v8i& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm_tie(v4i& x, v4i& y) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}

// F8: the fp8 path.  A tap's two 32-channel k-steps form one
// 64-deep v_mfma_f32_32x32x64_f8f6f4 (A = the tap's two resident weight
// fragments, B = the pixel's two channel-half fragments): 9 MFMAs per tile at
// twice the i8 cycles = the int8 MFMA time; pixel fragments one tap ahead.
// Epilogues: enc4_f8 with the residual decoded by v_cvt_f32_fp8.
template <bool F8>
__global__ __launch_bounds__(512, 1) void block_l1_kernel(BlockArgs a) {
  using Acc = typename std::conditional<F8, v16f, v16i>::type;
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: roles branch on SGPRs
  const int lr = lane & 31, lh = lane >> 5;
  const bool second = wave >= 4;  // conv2 wave
  int i0, J;
  xcd_chunk(a.N, i0, J);  // this workgroup's images: xcd_item(i0, 0 .. J-1)
  const int rows = J * LW;
  const int nphase = rows / RPH + 2;  // conv2 trails conv1 by 9 rows
  const unsigned lds32 = lds_addr32(lds);

  // Zero the intermediate ring (its padding units and zero row are never
  // written again) and the input ring's zero row.
  for (int i = tid; i < RING / 16; i += 512) *(v4i*)(lds + OFF_MID + 16 * i) = v4i{0, 0, 0, 0};
  for (int i = tid; i < 4 * PROW / 16; i += 512)
    *(v4i*)(lds + OFF_IN + (i >> 6) * PL + NR * PROW + 16 * (i & 63)) = v4i{0, 0, 0, 0};

  // Wave roles: conv (second), output-channel half h (oc h*32 .. h*32+31) and
  // job parity.  Per phase each conv has 7 jobs of 64 pixels per half; conv1
  // waves 0,1 take jobs 0,2,4,6 and waves 2,3 jobs 1,3,5; conv2 waves 4,5 take
  // 1,3,5 and 6,7 take 0,2,4,6 -- so the two waves of every SIMD (w, w+4)
  // share exactly 7 jobs.
  const int h = wave & 1, j0 = second ? 1 - ((wave >> 1) & 1) : (wave >> 1) & 1;

  // This wave's weights, resident in VGPRs: wr[ks] = A fragment of k-step ks
  // (tap ks/2, channels 32*(ks&1) + 16*lh ..) for output channel h*32 + lr.
  v4i wr[KS];
  const int8_t* ws = second ? a.w2 : a.w1;
  const int ol = h * 32 + lr;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int tap = ks >> 1, kk = ks & 1;
    wr[ks] = *(const v4i*)(ws + ol * 576 + tap * 64 + (((2 * kk + lh) ^ ((ol >> 2) & 3)) << 4));
  }
  // alpha/beta of this lane's 16 channels in the MFMA layout (oc h*32 + 8g + 4lh + e)
  float al[16], be[16];
  {
    const float* pa = second ? a.a2 : a.a1;
    const float* pb = second ? a.b2 : a.b1;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        al[4 * g4 + e] = pa[h * 32 + 8 * g4 + 4 * lh + e];
        be[4 * g4 + e] = pb[h * 32 + 8 * g4 + 4 * lh + e];
      }
  }

  // LDS-DMA of input row R into its ring slot: one piece per (row, plane),
  // lane i -> unit i of the plane row (pixel i-1; units 0 and 57..63 and rows
  // outside [0, rows) read zeros).  The row pointer and slot are wave-uniform
  // (SALU); per lane only the column/plane offset is added.
  auto row_src = [&](int R) -> const int8_t* {
    if (R < 0 || R >= rows) return nullptr;
    const int j = R / LW, r = R - j * LW;
    return a.x + ((size_t)xcd_item(i0, j) * LW + r) * (LW * LC);
  };
  const bool pix_lane = lane >= 1 && lane <= LW;
  auto dma_piece = [&](int R, int p) {
    const int8_t* rp = row_src(R);
    const int8_t* src = (rp && pix_lane) ? rp + (lane - 1) * LC + p * 16 : g_zero_b + (lane & 3) * 16;
    glds16_asm(src, lds32 + OFF_IN + p * PL + pos_mod(R, NR) * PROW);
  };

  for (int P = wave; P < 36; P += 8) dma_piece(P >> 2, P & 3);  // rows 0..8
  wait_vm0();
  __syncthreads();

  // Row bases of one lane's pixel: slot s0 holds the row above it (s0 + 1,
  // s0 + 2 the next two, mod NR); r = its image-local row.  ra[kh] = byte
  // address of unit `col` (= padded position of column col-1) in plane lh of
  // that row, or of the zero row.
  auto row_addrs = [&](int ring, int s0, int r, int col, bool valid, unsigned (&ra)[3]) {
    int sl = s0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      if (kh) {
        ++sl;
        if (sl == NR) sl = 0;
      }
      const bool rok = valid && (kh == 0 ? r > 0 : kh == 2 ? r < LW - 1 : true);
      ra[kh] = lds32 + ring + lh * PL + (rok ? sl : NR) * PROW + 16 * col;
    }
  };

  // One job: 32 oc x 64 pixels (two 32-pixel tiles) x 576 K, one
  // accumulation chain per tile (a dependent v_mfma_i32_32x32x32_i8 chain
  // issues at the full rate); pixel fragments are read two k-steps ahead.
  // k-step ks = tap (kh, kw), channel half kk: row base ra[kh], immediate
  // offset 16*kw + kk*2 planes.
  auto run_job = [&](const unsigned (&r0)[3], const unsigned (&r1)[3], Acc (&acc)[2]) {
    acc[0] = Acc{0};
    acc[1] = Acc{0};
    if constexpr (F8) {
      v8i bq[2][2];
      auto ld2 = [&](auto tc, int buf) {
        constexpr int tap = decltype(tc)::value, kh = tap / 3, kw = tap % 3;
        bq[buf][0] = cat8(ds_read16<16 * kw>(r0[kh]), ds_read16<16 * kw + 2 * PL>(r0[kh]));
        bq[buf][1] = cat8(ds_read16<16 * kw>(r1[kh]), ds_read16<16 * kw + 2 * PL>(r1[kh]));
      };
      ld2(std::integral_constant<int, 0>{}, 0);
      auto tstep = [&](auto tc) {
        constexpr int tap = decltype(tc)::value;
        if constexpr (tap + 1 < 9) ld2(std::integral_constant<int, tap + 1>{}, (tap + 1) & 1);
        wait_lgkm_tie8<tap + 1 < 9 ? 4 : 0>(bq[tap & 1][0], bq[tap & 1][1]);
        const v8i wa = cat8(wr[2 * tap], wr[2 * tap + 1]);
        acc[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wa, bq[tap & 1][0], acc[0], 0, 0, 0, 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wa, bq[tap & 1][1], acc[1], 0, 0, 0, 0, 0, 0);
      };
      static_for<0, 9>(tstep);
      return;
    } else {
    v4i bf[3][2];
    auto ld = [&](auto nc, int buf) {
      constexpr int n = decltype(nc)::value, tap = n >> 1, kh = tap / 3, kw = tap % 3;
      constexpr int off = 16 * kw + (n & 1) * 2 * PL;
      bf[buf][0] = ds_read16<off>(r0[kh]);
      bf[buf][1] = ds_read16<off>(r1[kh]);
    };
    ld(std::integral_constant<int, 0>{}, 0);
    ld(std::integral_constant<int, 1>{}, 1);
    auto step = [&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      if constexpr (ks + 2 < KS) ld(std::integral_constant<int, ks + 2>{}, (ks + 2) % 3);
      constexpr int younger = (ks + 2 < KS ? 2 : 0) + (ks + 1 < KS ? 2 : 0);
      wait_lgkm_tie<younger>(bf[ks % 3][0], bf[ks % 3][1]);
      acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], bf[ks % 3][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[ks], bf[ks % 3][1], acc[1], 0, 0, 0);
    };
    static_for<0, KS>(step);
    }
  };

  // Epilogue of one 32 oc x 32 px tile in the MFMA layout (lane: pixel lr,
  // channels h*32 + 8g + 4lh + e) -> 16 contiguous channels (h*32 + 16lh ..)
  // of the pixel.  rs: the residual's 16 bytes in that store layout (conv2).
  // Pairs of elements go through v_pk_fma_f32 / v_pk_add_f32 (per-component
  // IEEE fma / add: bit-identical to the scalar sequence).
  auto epilogue = [&](const Acc& acc, bool res, v4i rs) -> v4i {
    if constexpr (F8) {
      unsigned rg[4] = {0, 0, 0, 0};
      if (res) {  // store layout -> MFMA layout (e4m3 bytes, decoded below)
        unsigned rr[4] = {(unsigned)rs[0], (unsigned)rs[1], (unsigned)rs[2], (unsigned)rs[3]};
        swap32(rr[0], rr[1]);
        swap32(rr[2], rr[3]);
        rg[0] = rr[0];
        rg[1] = rr[2];
        rg[2] = rr[1];
        rg[3] = rr[3];
      }
      unsigned qv[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float ac[4] = {acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]};
        qv[g4] = res ? epi4_res_f8(ac, al + 4 * g4, be + 4 * g4, rg[g4], a.s_res, 0.f)
                     : epi4_f8(ac, al + 4 * g4, be + 4 * g4, 0.f);
      }
      return mfma_to_store16(qv[0], qv[1], qv[2], qv[3]);
    }
    unsigned rg[4] = {0, 0, 0, 0};
    if (res) {  // store layout -> MFMA layout
      unsigned rr[4] = {(unsigned)rs[0], (unsigned)rs[1], (unsigned)rs[2], (unsigned)rs[3]};
      swap32(rr[0], rr[1]);
      swap32(rr[2], rr[3]);
      rg[0] = rr[0] ^ 0x80808080u;  // biased: int8 v = ubyte(v ^ 0x80) - 128, exact in fp32
      rg[1] = rr[2] ^ 0x80808080u;
      rg[2] = rr[1] ^ 0x80808080u;
      rg[3] = rr[3] ^ 0x80808080u;
    }
    const f2 M2 = {12582912.0f, 12582912.0f}, sr2 = {a.s_res, a.s_res}, m128 = {-128.f, -128.f};
    unsigned qv[4];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      f2 y[2];
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const int e = 4 * g4 + 2 * p2;
        y[p2] = __builtin_elementwise_fma(f2{(float)acc[e], (float)acc[e + 1]}, f2{al[e], al[e + 1]},
                                          f2{be[e], be[e + 1]});
        if (res) {
          const f2 rv = f2{(float)((rg[g4] >> (16 * p2)) & 0xffu), (float)((rg[g4] >> (16 * p2 + 8)) & 0xffu)} + m128;
          y[p2] = __builtin_elementwise_fma(rv, sr2, y[p2]);
        }
        y[p2] = f2{__builtin_amdgcn_fmed3f(y[p2][0], 0.f, 127.f), __builtin_amdgcn_fmed3f(y[p2][1], 0.f, 127.f)} + M2;
      }
      const unsigned u0 = __float_as_uint(y[0][0]), u1 = __float_as_uint(y[0][1]);
      const unsigned u2 = __float_as_uint(y[1][0]), u3 = __float_as_uint(y[1][1]);
      qv[g4] = __builtin_amdgcn_perm(u1, u0, 0x0c0c0400u) | __builtin_amdgcn_perm(u3, u2, 0x04000c0cu);
    }
    return mfma_to_store16(qv[0], qv[1], qv[2], qv[3]);
  };

  // pixel of tile t of job j: phase-relative row ro (0..7) and column
  auto pix_of = [&](int j, int t, int& ro, int& col) {
    const int px = j * 64 + t * 32 + lr;
    ro = (px * 1171) >> 16;  // px / 56 for px < 448
    col = px - ro * LW;
  };

  BT_DECL;
  for (int g = 0; g < nphase; ++g) {
    const int G = g * RPH;
    if (!second) {
      // conv1 waves also stream the next phase's input rows [G+9, G+17): wave
      // c issues plane c of all 8 rows, two pieces per job, so only conv1
      // waves ever wait on LDS-DMA.
      int kp = 0;
      auto pieces = [&](int n) {
        for (int e = 0; e < n && kp < 8; ++e, ++kp) dma_piece(G + 9 + kp, wave);
      };
      if (G < rows && BL1_TEST != 2) {
        // slots of rows G-1 (taps) and G (output), image-local row of G
        const int S_in = pos_mod(G - 1, NR), S_mid = G % NR, r0 = G % LW;
        for (int j = j0; j < 7; j += 2) {
          BT(0);
          pieces(2);
          BT(5);
          unsigned ra[2][3], wa[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            int ro, col;
            pix_of(j, t, ro, col);
            int s0 = S_in + ro;
            if (s0 >= NR) s0 -= NR;
            row_addrs(OFF_IN, s0, r0 + ro, col, true, ra[t]);
            int sm = S_mid + ro;
            if (sm >= NR) sm -= NR;
            wa[t] = OFF_MID + (2 * h + lh) * PL + sm * PROW + 16 * (col + 1);
          }
          Acc acc[2];
          BT(0);
          run_job(ra[0], ra[1], acc);
          BT(1);
#pragma unroll
          for (int t = 0; t < 2; ++t) *(v4i*)(lds + wa[t]) = epilogue(acc[t], false, v4i{0, 0, 0, 0});
          BT(2);
        }
      }
      if (G + 9 < rows) pieces(8);
      BT(3);
      wait_vm0();  // this phase's DMA has landed
    } else {
      // output rows start at global row G-9: MID slot of the row above it,
      // its image-local row and image ordinal
      const int S_mid = pos_mod(G - 10, NR), rr0 = pos_mod(G - 9, LW), jm0 = (G - 9 - rr0) / LW;
      // per job: tap rows, output pointers and the residual (the block
      // input, 16 channels of this lane, loaded before the job's MFMAs and
      // awaited after them; conv2 waves issue no LDS-DMA, so the wait covers
      // only these loads and the previous job's stores).  The loads land in
      // registers no other code touches before the tied wait: no copies of
      // in-flight registers.
      for (int j = j0; j < 7; j += 2) {
        const int R0 = G - 9 + (j * 64) / LW, R1 = G - 9 + (j * 64 + 63) / LW;
        if (R1 < 0 || R0 >= rows || BL1_TEST == 1) continue;  // no pixel of this job exists (wave-uniform)
        unsigned ra[2][3];
        int8_t* dst[2];
        v4i rq[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          int ro, col;
          pix_of(j, t, ro, col);
          const int R = G - 9 + ro;
          const bool valid = R >= 0 && R < rows;
          int r = rr0 + ro, jm = jm0;
          if (r >= LW) {
            r -= LW;
            ++jm;
          }
          int s0 = S_mid + ro;
          if (s0 >= NR) s0 -= NR;
          row_addrs(OFF_MID, s0, r, col, valid, ra[t]);
          const size_t pix = valid ? ((size_t)xcd_item(i0, jm) * LW + r) * LW + col : 0;
          if constexpr (BL1_TEST == 7)
            rq[t] = v4i{0, 0, 0, 0};
          else
            rq[t] = gload16_untracked(a.x + pix * LC + h * 32 + lh * 16);
          dst[t] = valid ? a.y + pix * LC + h * 32 + lh * 16 : g_trash_b + lane * 16;
        }
        Acc acc[2];
        BT(0);
        run_job(ra[0], ra[1], acc);
        BT(1);
        wait_vm_tie<0>(rq[0], rq[1]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          int8_t* d = dst[t];
          if constexpr (BL1_TEST == 8) d = g_trash_b + lane * 16;
          *(v4i*)d = epilogue(acc[t], true, rq[t]);
        }
        BT(2);
      }
      BT(3);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): intermediate rows written (vmcnt untouched)
    __builtin_amdgcn_s_barrier();
    BT(4);
  }
  BT_STORE();
  wait_vm0();
}

// ---- int8: software-pipelined jobs -------------------------------------
// The same phases, rings, resident weights and epilogue arithmetic as
// block_l1_kernel, with one-tile jobs (32 oc x 32 px x 576 K: ONE
// accumulation chain of 18 v_mfma_i32_32x32x32_i8) and the epilogue of job
// k - 1 interleaved with the MFMA chain of job k (two accumulator sets), so a
// wave's requantisation VALU hides in its own MFMA gaps instead of leaving
// the SIMD's matrix pipe to the partner wave.  A phase's 14 tiles per oc half
// are dealt by parity (tile t = par + 2k, k < 7), so every SIMD (waves w and
// w + 4: one conv1 and one conv2 wave of the same oc half and parity) gets 7
// conv1 and 7 conv2 jobs.  Measured before: the SIMD pairs' 4 + 3 two-tile
// jobs left the conv1 waves 30-40 % of the phase at the barrier while the
// conv2 waves ran their VALU-heavy residual epilogues serially.
// Untracked fragment reads never stay in flight across a branch or a loop
// edge (each job reads its own first two k-steps); the residual is a
// compiler-tracked load (conv2 waves issue no LDS-DMA, so the compiler's
// vmcnt arithmetic is exact for them).
// The requantisation runs between the MFMAs of the next job: scalar FMAs
// (device_common.h epi4_relu / epi4_res_relu).
#define DLQ_L1_EPI epi4_relu
#define DLQ_L1_EPI_RES epi4_res_relu
template <bool SECOND>
__device__ __forceinline__ void block_l1_sp_role(const BlockArgs& a, int8_t* lds, unsigned lds32, int wave, int rows,
                                                 int nphase) {
  const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5;
  int i0, nimg;
  xcd_chunk(a.N, i0, nimg);  // this workgroup's images: xcd_item(i0, 0 .. nimg-1)
  const int h = wave & 1, par = (wave >> 1) & 1;  // output-channel half, tile parity
  v4i wr[KS];
  const int8_t* ws = SECOND ? a.w2 : a.w1;
  const int ol = h * 32 + lr;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int tap = ks >> 1, kk = ks & 1;
    wr[ks] = *(const v4i*)(ws + ol * 576 + tap * 64 + (((2 * kk + lh) ^ ((ol >> 2) & 3)) << 4));
  }
  float al[16], be[16];
  {
    const float* pa = SECOND ? a.a2 : a.a1;
    const float* pb = SECOND ? a.b2 : a.b1;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        al[4 * g4 + e] = pa[h * 32 + 8 * g4 + 4 * lh + e];
        be[4 * g4 + e] = pb[h * 32 + 8 * g4 + 4 * lh + e];
      }
  }
  auto row_src = [&](int R) -> const int8_t* {
    if (R < 0 || R >= rows) return nullptr;
    const int j = R / LW, r = R - j * LW;
    return a.x + ((size_t)xcd_item(i0, j) * LW + r) * (LW * LC);
  };
  const bool pix_lane = lane >= 1 && lane <= LW;
  auto dma_piece = [&](int R, int p) {
    const int8_t* rp = row_src(R);
    const int8_t* src = (rp && pix_lane) ? rp + (lane - 1) * LC + p * 16 : g_zero_b + (lane & 3) * 16;
    glds16_asm(src, lds32 + OFF_IN + p * PL + pos_mod(R, NR) * PROW);
  };
  for (int P = wave; P < 36; P += 8) dma_piece(P >> 2, P & 3);  // rows 0..8
  wait_vm0();
  __syncthreads();

  auto row_addrs = [&](int ring, int s0, int r, int col, bool valid, unsigned (&ra)[3]) {
    int sl = s0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      if (kh) {
        ++sl;
        if (sl == NR) sl = 0;
      }
      const bool rok = valid && (kh == 0 ? r > 0 : kh == 2 ? r < LW - 1 : true);
      ra[kh] = lds32 + ring + lh * PL + (rok ? sl : NR) * PROW + 16 * col;
    }
  };
  // one epilogue group (4 values: MFMA-layout register group g4) of a finished tile
  auto epi_group = [&](const v16i& acc, int g4, const unsigned (&rg)[4]) -> unsigned {
    const int ac[4] = {acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]};
    if constexpr (SECOND)
      return DLQ_L1_EPI_RES(ac, al + 4 * g4, be + 4 * g4, rg[g4], a.s_res);
    else
      return DLQ_L1_EPI(ac, al + 4 * g4, be + 4 * g4);
  };
  // store layout -> MFMA layout
  auto res_regs = [&](const v4i& rs, unsigned (&rg)[4]) {
    unsigned rr[4] = {(unsigned)rs[0], (unsigned)rs[1], (unsigned)rs[2], (unsigned)rs[3]};
    swap32(rr[0], rr[1]);
    swap32(rr[2], rr[3]);
    rg[0] = rr[0];
    rg[1] = rr[2];
    rg[2] = rr[1];
    rg[3] = rr[3];
  };

  // (conv2's residual is re-read from global memory, an L2 hit mostly; the
  // variant that read it from the LDS input ring cut the launch's HBM bytes
  // 141 -> 102 MB but ran 1.9 us slower: round-4 DESIGN.md §6, commit e071b4a)
  // the conv2 waves are the critical path (residual epilogues): they win
  // the SIMD's issue arbitration against their conv1 partner, which then
  // spends less of the phase waiting at the barrier
#ifndef DLQ_L1_PRIOJ
#define DLQ_L1_PRIOJ 6  // measured: 5 of 7 jobs 64.2-64.5 us, all 7 66.0, none 65.9-67.4 (tools/probe/block_l1_sp_stamps.hip); with the DMA inside the conv1 chains 6 of 7: median 61.4 vs 62.3 (5) and 62.0 (4) us, four A/B rounds
#endif
  BT_DECL;
  for (int g = 0; g < nphase; ++g) {
    const int G = g * RPH;
    const int S_in = pos_mod(G - 1, NR), S_mid1 = G % NR, r01 = G % LW;
    const int S_mid2 = pos_mod(G - 10, NR), rr0 = pos_mod(G - 9, LW), jm0 = (G - 9 - rr0) / LW;
    // this phase's jobs k = kb .. ke-1 (tile t = par + 2k; wave-uniform)
    // The last phase's conv2 takes 9 rows (16 tiles, k < 8): its ninth row
    // needs intermediate rows up to the image's last, written the phase
    // before, so no phase is left for that one row.
    int kb = 0, ke = 0;
    const bool lastp = g == nphase - 1;
    if constexpr (!SECOND) {
      if (G < rows) ke = 7;
    } else if (!lastp && G - 9 >= 0 && G - 2 < rows) {  // every output row of the phase exists
      ke = 7;
    } else {
      for (int k = 0; k < (lastp ? 8 : 7); ++k) {  // output rows G-9 + (32t .. 32t+31) / 56 must reach [0, rows)
        const int t = par + 2 * k;
        const int R0 = G - 9 + (t * 32) / LW, R1 = G - 9 + (t * 32 + 31) / LW;
        const bool any = R1 >= 0 && R0 < rows;
        if (any && ke == kb) {
          kb = k;
          ke = k + 1;
        } else if (any) {
          ke = k + 1;
        }
      }
    }
    // conv1 waves stream input rows G+9 .. G+16 (plane = wave), two pieces
    // per job over the first four jobs
    int dma_left = (!SECOND && G + 9 < rows) ? 8 : 0, dma_row = 0;
    auto dma_some = [&](int n) {
      for (int e = 0; e < n && dma_left > 0; ++e, --dma_left, ++dma_row) dma_piece(G + 9 + dma_row, wave);
    };

    // per job: tap row bases, then (conv1) the intermediate slot offset or
    // (conv2) the residual and the output pointer
    struct Job {
      unsigned ra[3];
      unsigned wa;
      v4i rq;
      int8_t* dst;
    };
    auto setup = [&](int k, Job& jb) {
      const int t = par + 2 * k;
      const int px = t * 32 + lr;
      const int ro = (px * 1171) >> 16;  // px / 56 for px < 512
      const int col = px - ro * LW;
      if constexpr (!SECOND) {
        int s0 = S_in + ro;
        if (s0 >= NR) s0 -= NR;
        row_addrs(OFF_IN, s0, r01 + ro, col, true, jb.ra);
        int sm = S_mid1 + ro;
        if (sm >= NR) sm -= NR;
        jb.wa = OFF_MID + (2 * h + lh) * PL + sm * PROW + 16 * (col + 1);
      } else {
        const int R = G - 9 + ro;
        const bool valid = R >= 0 && R < rows;
        int r = rr0 + ro, jm = jm0;
        if (r >= LW) {
          r -= LW;
          ++jm;
        }
        int s0 = S_mid2 + ro;
        if (s0 >= NR) s0 -= NR;
        row_addrs(OFF_MID, s0, r, col, valid, jb.ra);
        const size_t pix = valid ? ((size_t)xcd_item(i0, jm) * LW + r) * LW + col : 0;
        jb.rq = *(const v4i*)(a.x + pix * LC + h * 32 + lh * 16);
        jb.dst = valid ? a.y + pix * LC + h * 32 + lh * 16 : g_trash_b + lane * 16;
      }
    };
    auto finish = [&](const v4i& o, const Job& jb) {
      if constexpr (SECOND)
        *(v4i*)jb.dst = o;
      else
        *(v4i*)(lds + jb.wa) = o;
    };
    v16i acc[2];
    Job job[2];
    // job k in set A (acc[A], job[A]); with PREV, job k-1 (set 1 - A) is
    // requantised and stored between the chain's MFMAs
    auto run = [&](auto ac, auto pc, int k) {
      constexpr int A = decltype(ac)::value, E = 1 - A;
      constexpr bool PREV = decltype(pc)::value;
      if constexpr (SECOND) {  // the first DLQ_L1_PRIOJ jobs of a phase at priority 1
        if (k - kb == 0) __builtin_amdgcn_s_setprio(DLQ_L1_PRIOJ > 0 ? 1 : 0);
        if (k - kb == DLQ_L1_PRIOJ) __builtin_amdgcn_s_setprio(0);
      }
      setup(k, job[A]);
      v4i bf[3];
      auto ld = [&](auto nc, int buf) {
        constexpr int n = decltype(nc)::value, tap = n >> 1, kh = tap / 3, kw = tap % 3;
        constexpr int off = 16 * kw + (n & 1) * 2 * PL;
        bf[buf] = ds_read16<off>(job[A].ra[kh]);
      };
      ld(std::integral_constant<int, 0>{}, 0);
      ld(std::integral_constant<int, 1>{}, 1);
      unsigned rg[4] = {0, 0, 0, 0}, qv[4] = {0, 0, 0, 0};
      acc[A] = v16i{0};
      auto step = [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s + 2 < KS) ld(std::integral_constant<int, s + 2>{}, (s + 2) % 3);
        if constexpr (PREV) {
          if constexpr (SECOND && s == 1) res_regs(job[E].rq, rg);
          if constexpr (s == 3 || s == 6 || s == 9 || s == 12) qv[(s - 3) / 3] = epi_group(acc[E], (s - 3) / 3, rg);
          if constexpr (s == 14) finish(mfma_to_store16(qv[0], qv[1], qv[2], qv[3]), job[E]);
        }
        // younger LDS ops than this k-step's read: the (up to) two prefetches,
        // plus at most one intermediate-ring write (waiting for it is harmless)
        constexpr int young = (s + 2 < KS ? 2 : s + 1 < KS ? 1 : 0);
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(bf[s % 3]) : "n"(young) : "memory");
        acc[A] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wr[s], bf[s % 3], acc[A], 0, 0, 0);
        // conv1 waves: the job's two input-ring pieces (first four jobs of a
        // phase) issue after the chain's 2nd and 4th MFMAs, beside the matrix
        // work instead of ahead of it (median of five A/B rounds on one box:
        // 63.3 -> 62.5 us per launch)
        if constexpr (!SECOND && (s == 1 || s == 3)) {
          if (k - kb < 4) dma_some(1);
        }
      };
      static_for<0, KS>(step);
    };
    auto final_epi = [&](auto ac, const v4i& rq) {  // the phase's last job, after its chain
      constexpr int A = decltype(ac)::value;
      unsigned rg[4] = {0, 0, 0, 0}, qv[4];
      if constexpr (SECOND) res_regs(rq, rg);
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) qv[g4] = epi_group(acc[A], g4, rg);
      finish(mfma_to_store16(qv[0], qv[1], qv[2], qv[3]), job[A]);
    };
    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, 1> I1;
    const std::integral_constant<bool, false> NOPREV;
    const std::integral_constant<bool, true> WPREV;
    BT(0);
    if (ke > kb) {
      run(I0, NOPREV, kb);
      int k = kb + 1;
      for (; k + 1 < ke; k += 2) {
        run(I1, WPREV, k);
        run(I0, WPREV, k + 1);
      }
      if (k < ke) {  // an odd job left: it runs in set 1, the last epilogue is set 1's
        run(I1, WPREV, k);
        final_epi(I1, job[1].rq);
      } else {
        final_epi(I0, job[0].rq);
      }
    }
    BT(1);
    // a phase of fewer than DLQ_L1_PRIOJ jobs never reached the lowering
    // above: every phase starts from priority 0
    if constexpr (SECOND) __builtin_amdgcn_s_setprio(0);
    if constexpr (!SECOND) {
      dma_some(8);
      // the last phase has no conv1 jobs: the idle conv1 waves pull the next
      // launch's first weight stages into the input ring (read by nothing now)
      if (lastp) prefetch_next(a.pf, wave, 4, lds32 + OFF_IN);
      wait_vm0();  // this phase's DMA has landed
    }
    BT(2);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): intermediate rows written (vmcnt untouched)
    __builtin_amdgcn_s_barrier();
    BT(3);
  }
  BT_STORE();
  wait_vm0();
}

__global__ __launch_bounds__(512, 1) void block_l1_sp_kernel(BlockArgs a) {
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int i0, J;
  xcd_chunk(a.N, i0, J);  // this workgroup's images (device_common.h xcd_chunk)
  const int rows = J * LW;
  const int nphase = rows / RPH + 1;  // conv2 trails conv1 by 9 rows; its last phase takes 9
  for (int i = tid; i < RING / 16; i += 512) *(v4i*)(lds + OFF_MID + 16 * i) = v4i{0, 0, 0, 0};
  for (int i = tid; i < 4 * PROW / 16; i += 512)
    *(v4i*)(lds + OFF_IN + (i >> 6) * PL + NR * PROW + 16 * (i & 63)) = v4i{0, 0, 0, 0};
  if (wave >= 4)
    block_l1_sp_role<true>(a, lds, lds_addr32(lds), wave, rows, nphase);
  else
    block_l1_sp_role<false>(a, lds, lds_addr32(lds), wave, rows, nphase);
}

int num_cus_b() {
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

bool block_l1_shape(int C, int OC, int H, int W) { return C == LC && OC == LC && H == LW && W == LW; }

hipError_t launch_block_l1(const int8_t* x, int N, const int8_t* w1, const float* a1, const float* b1,
                           const int8_t* w2, const float* a2, const float* b2, float s_res, int8_t* y,
                           hipStream_t s, bool f8, const Prefetch* pf) {
  if (N <= 0) return hipSuccess;
  BlockArgs a{x, y, w1, w2, a1, b1, a2, b2, s_res, N, pf ? *pf : Prefetch{}};
  int grid = num_cus_b();
  {  // knob "l1_grid" (DLQ_L1_GRID, dlq_set_knob): several images per workgroup
    const int g = g_knob_l1_grid.load(std::memory_order_relaxed);
    if (g > 0 && g < grid) grid = g;
  }
  if (f8)
    hipLaunchKernelGGL(block_l1_kernel<true>, dim3(N < grid ? N : grid), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL(block_l1_sp_kernel, dim3(N < grid ? N : grid), dim3(512), 0, s, a);
  return hipGetLastError();
}

}  // namespace dlq
