// gemm.hip -- dlq_gemm_s8s8s32: C[M][N] (int32) = A[M][K] . B[K][N] (int8),
// row-major, any M, N, K: the int8 replacement of the reference's exported
// sgemm_tiled (RK/kernels/sgemm_tiled.cu:5-46, called by
// conv2d_nchw_im2col_gemm RK/runtime/infer_e2e.cu:129-133 with A = OIHW
// weights [OC][IC*kH*kW], B = im2col [IC*kH*kW][OH*OW]).  int32 sums are
// exact, so any k order gives the reference's accumulators bit for bit.
//
// Two kernels.  K % 16 == N % 16 == 0 (16-byte aligned bases): the LDS-DMA
// kernel below (gemm_s8s8s32_k128_kernel, K = 128 per stage, tile 256 x 256,
// 256 x 128 or 128 x 128 chosen by shape).  Otherwise the register-staged
// kernel: tile 256 x 256 per 512-thread workgroup (8 waves = 2 (M) x 4 (N), each 128 x
// 64 = 4 x 2 v_mfma_i32_32x32x32_i8 tiles), K = 64 per stage, double-buffered
// LDS (2 x 40 KiB), one barrier per stage; global loads run two stages ahead
// in two register sets, so each has two stages of MFMAs to land.
//  * A rows are K-contiguous, as the MFMA wants: 16-byte loads straight into
//    LDS rows [m][64 k].
//  * B is N-contiguous in memory but the MFMA's B operand is K-contiguous per
//    column: each thread loads a 4 (k) x 8 (n) block as four 8-byte row loads
//    (a wave covers 2 KiB of contiguous rows), transposes it in registers with
//    v_perm_b32 (16 perms) and stores 8 column dwords to LDS rows [n][64 k].
//  * LDS row pitch 80 B (5 units): the 16 rows a ds_read_b128 lane group
//    reads fall on 16 distinct bank quads.
//  * blockIdx -> tile is XCD-aware: each XCD runs a contiguous run of tiles
//    (same A row block) so A and B panels are reused from its L2.
// Edge tiles and unaligned leading dimensions take byte loads with bounds
// checks (zeros outside), interior aligned tiles vector loads.
#include "device_common.h"

namespace dlq {
namespace {

constexpr int GT = 256;  // tile M = tile N
constexpr int GK = 64;   // K per stage
constexpr int GP = 80;   // LDS row pitch in bytes
constexpr int GSLOT = 2 * GT * GP;  // A rows then B rows

__device__ __forceinline__ unsigned ld_bytes(const int8_t* p, int avail) {  // up to 4 bytes, zero-filled
  unsigned v = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (e < avail) v |= (unsigned)(uint8_t)p[e] << (8 * e);
  return v;
}

// BT: B is supplied transposed, Bt[N][K] (K-contiguous rows, loaded and
// staged exactly as A's rows: no register transpose).
template <bool BT>
__global__ __launch_bounds__(512, 1) void gemm_s8s8s32_generic_kernel(const int8_t* __restrict__ A,
                                                             const int8_t* __restrict__ B, int32_t* __restrict__ C,
                                                             int M, int N, int K, int nbn, int aligned) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * GSLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int l = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (l / nbn) * GT, n0 = (l % nbn) * GT;
  const int wm = wave >> 2, wn = wave & 3;
  const bool full_mn = aligned && m0 + GT <= M && n0 + GT <= N;
  // A: rows (tid >> 2) and +128, 16-byte chunk tid & 3; B: 8 columns 8 * (tid & 31), rows 4 * (tid >> 5) .. +3
  const int a_row = tid >> 2, a_ch = tid & 3;
  const int b_cg = tid & 31, b_rq = tid >> 5;
  // Two stages of global loads in flight in registers: set (s & 1) holds
  // stage s + 1 while stage s + 2's loads are issued into the other set, so
  // each load has two stages of MFMAs to land before its LDS write.
  v4i ra[2][2];
  unsigned rb[2][4][2];
  v4i rbt[2][2];  // BT: rows n0 + a_row (+128), chunk a_ch

  auto gload = [&](int k0, int set) {
    if (full_mn && k0 + GK <= K) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        ra[set][p] = *(const v4i*)(A + (size_t)(m0 + a_row + 128 * p) * K + k0 + a_ch * 16);
      if constexpr (BT) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          rbt[set][p] = *(const v4i*)(B + (size_t)(n0 + a_row + 128 * p) * K + k0 + a_ch * 16);
        return;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint2 v = *(const uint2*)(B + (size_t)(k0 + 4 * b_rq + r) * N + n0 + 8 * b_cg);
        rb[set][r][0] = v.x;
        rb[set][r][1] = v.y;
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int m = m0 + a_row + 128 * p, k = k0 + a_ch * 16;
      const int8_t* src = A + (size_t)m * K + k;
#pragma unroll
      for (int w = 0; w < 4; ++w) ra[set][p][w] = (int)(m < M ? ld_bytes(src + 4 * w, K - k - 4 * w) : 0u);
    }
    if constexpr (BT) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int n = n0 + a_row + 128 * p, k = k0 + a_ch * 16;
        const int8_t* src = B + (size_t)n * K + k;
#pragma unroll
        for (int w = 0; w < 4; ++w) rbt[set][p][w] = (int)(n < N ? ld_bytes(src + 4 * w, K - k - 4 * w) : 0u);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 4 * b_rq + r, n = n0 + 8 * b_cg;
      const int8_t* src = B + (size_t)k * N + n;
      rb[set][r][0] = k < K ? ld_bytes(src, N - n) : 0u;
      rb[set][r][1] = k < K ? ld_bytes(src + 4, N - n - 4) : 0u;
    }
  };
  auto lstore = [&](int slot, int set) {
    int8_t* la = lds + slot * GSLOT;
    int8_t* lb = la + GT * GP;
#pragma unroll
    for (int p = 0; p < 2; ++p) *(v4i*)(la + (a_row + 128 * p) * GP + a_ch * 16) = ra[set][p];
    if constexpr (BT) {
#pragma unroll
      for (int p = 0; p < 2; ++p) *(v4i*)(lb + (a_row + 128 * p) * GP + a_ch * 16) = rbt[set][p];
      return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // 4 x 4 byte transpose: rows k..k+3 -> column dwords
      const unsigned t0 = __builtin_amdgcn_perm(rb[set][1][h], rb[set][0][h], 0x05010400u);
      const unsigned t1 = __builtin_amdgcn_perm(rb[set][1][h], rb[set][0][h], 0x07030602u);
      const unsigned t2 = __builtin_amdgcn_perm(rb[set][3][h], rb[set][2][h], 0x05010400u);
      const unsigned t3 = __builtin_amdgcn_perm(rb[set][3][h], rb[set][2][h], 0x07030602u);
      const unsigned d[4] = {__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
                             __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u)};
#pragma unroll
      for (int c = 0; c < 4; ++c) *(unsigned*)(lb + (8 * b_cg + 4 * h + c) * GP + 4 * b_rq) = d[c];
    }
  };
  auto compute = [&](int slot, v16i (&acc)[4][2]) {
    const int8_t* la = lds + slot * GSLOT;
    const int8_t* lb = la + GT * GP;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v4i fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *(const v4i*)(la + (wm * 128 + i * 32 + lr) * GP + ks * 32 + lh * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *(const v4i*)(lb + (wn * 64 + j * 32 + lr) * GP + ks * 32 + lh * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  v16i acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = v16i{0};
  const int nst = (K + GK - 1) / GK;
  gload(0, 0);
  if (nst > 1) gload(GK, 1);
  lstore(0, 0);
  __syncthreads();
  // iteration s: stage s + 2's loads into register set s & 1 (its stage s
  // went to LDS one iteration ago), stage s from LDS slot s & 1, then stage
  // s + 1 (set (s + 1) & 1, landed during this stage) into the other slot.
  int s = 0;
  for (; s + 1 < nst; s += 2) {  // unrolled by two so the register sets are compile-time
    if (s + 2 < nst) gload((s + 2) * GK, 0);
    compute(0, acc);
    lstore(1, 1);
    __syncthreads();
    if (s + 3 < nst) gload((s + 3) * GK, 1);
    compute(1, acc);
    if (s + 2 < nst) lstore(0, 0);
    __syncthreads();
  }
  if (s < nst) compute(0, acc);  // odd stage count: the last stage sits in slot 0
  // D reg r, lane (lr, lh): row (r & 3) + 8 (r >> 2) + 4 lh, column lr of the 32 x 32 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M && n < N) C[(size_t)m * N + n] = acc[i][j][r];
      }
    }
}


// ---- aligned operands (K % 16 == 0, N % 16 == 0, 16-byte aligned bases):
// both tiles stream by LDS-DMA, K = 128 per stage through two slots.  Stage
// s + 1 is issued after the barrier that opens stage s (every wave has
// left stage s - 1's slot by then), one piece after each of k-step 0's 8
// MFMAs, so its 64 KB land during stage s's 32 MFMAs per wave and the matrix
// pipe runs while the pieces issue (issued back to back after the barrier:
// 8192^3 1598-1635 vs 1652-1684 TOPS, 50176 x 256 x 2304 1361-1372 vs
// 1447-1463, three alternating runs on one box).  (A 4-slot ring of K = 64 stages, three ahead, measured
// 6-12 % slower on one box: 8192^3 1547 vs 1646 TOPS, 4096^3 1648 vs 1852,
// 50176 x 256 x 2304 1239 vs 1345 -- twice the barriers per K.)
//  * A image: row m = 128 K bytes, chunk c at m*128 + 16*(c ^ ((m >> 1) & 7)):
//    a ds_read_b128 lane group's 16 rows (8 even, 8 odd) on 16 bank quads.
//  * B image: K rows of 256 N bytes as loaded (no register transpose): chunk b
//    of row k at k*256 + 16*(b ^ 2(k & 7)).  The MFMA B fragment (16 K bytes
//    of one column) is two ds_read_b64_tr_b8: per 16-lane group, lane 2q + p
//    addresses row q (of 8), columns 8p .. 8p+7, and lane i receives column
//    i's 8 row bytes (probed on gfx950); the XOR puts a 32-lane half's 8 rows
//    x 32 columns on 64 distinct banks.
//  * The swizzles are applied on the global side: DMA lane t of a piece
//    fetches the global chunk whose swizzled LDS position is t.

__device__ __attribute__((aligned(64))) int8_t g_zero_gemm[64];


constexpr int GK2 = 128;

// Tile TM x TN per workgroup of WM x WN waves, each wave MI x NJ MFMA tiles
// (32 x 32); TM = 32 WM MI, TN = 32 WN NJ.  Per stage K = 128: TM / 8 A
// pieces (8 rows x 128 K bytes each) and TNP / 8 B pieces (1024 / TNP K rows
// x TNP bytes each), dealt to the waves round-robin (a wave whose last slot
// index passes the piece count issues nothing there: wave-uniform).  TNP =
// TN but 256 for TN = 224 (7 MFMA columns): the B image keeps the 256-byte
// row pitch and swizzle, its two spare chunks per row read zeros.
//  * A image: row m = 128 K bytes, chunk c at m*128 + 16*(c ^ ((m >> 1) & 7)).
//  * B image: K rows of TN bytes as loaded: chunk b of row k at k*TN +
//    16*(b ^ swz(k)), swz(k) = 2(k & 7) for TN = 256 and 2((k >> 1) & 3) for
//    TN = 128 -- either way a ds_read_b64_tr_b8 half-wave's 8 rows x 32
//    columns fall on 64 distinct banks, and swz(k + 8) = swz(k).
template <int TN>
__device__ __forceinline__ int bswz(int k) {
  return TN == 256 ? 2 * (k & 7) : 2 * ((k >> 1) & 3);
}
template <int TN>
constexpr int b_pitch() {  // B image row pitch (NN) / staged rows (NT)
  return TN == 224 ? 256 : TN;
}

// BT: B supplied transposed (Bt[N][K]): its tile is staged and read exactly
// as A's (rows of 128 K bytes, chunk c at n*128 + 16*(c ^ ((n >> 1) & 7))),
// one ds_read_b128 per B fragment instead of two ds_read_b64_tr_b8.
//
// One tile's K stages [sb, se) into acc (zeroed here).  Loads past
// min(K, 128 se) read zeros.  Returns with every DMA of the range landed.
// (A stream-K split over [sb, se) ranges, int32 partials handed to the
// last contributor through write-through stores, was measured bit-exact but
// slower on every shape: DESIGN.md §6, profiles/r05_gemm_streamk.txt.)
template <int WM, int WN, int MI, int NJ, bool BT>
__device__ __forceinline__ void k128_tile(const int8_t* __restrict__ A, const int8_t* __restrict__ B, int M, int N,
                                          int K, int m0, int n0, int sb, int se, int8_t* lds,
                                          v16i (&acc)[MI][NJ]) {
  constexpr int NW = WM * WN, TM = 32 * WM * MI, TN = 32 * WN * NJ, TNP = b_pitch<TN>();
  constexpr int SA = TM * GK2, SLOT = SA + GK2 * TNP;  // slot: A image, then B image
  constexpr int PA = TM / 8, PB = TNP / 8, NP = PA + PB, PPW = (NP + NW - 1) / NW;  // pieces: A, B, per wave
  constexpr int CPR = TNP / 16;  // B chunks per K row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const unsigned lds32 = lds_addr32(lds);
  const int kend = K < se * GK2 ? K : se * GK2;

  // the zero source once, in SGPRs (re-derived per piece it cost an
  // s_load + lgkmcnt(0) wait beside the MFMAs)
  const int8_t* zsrc = g_zero_gemm;
  asm volatile("" : "+s"(zsrc));
  auto issue_r = [&](int st, int r) {  // this wave's piece r of stage st
    const int k0 = st * GK2;
    const unsigned slot = lds32 + (st & 1) * SLOT;
    const int pc = wave + NW * r;
    if (NP % NW != 0 && pc >= NP) return;  // wave-uniform: no piece in this slot
    if (pc < PA) {
      const int m = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((m >> 1) & 7), k = k0 + 16 * c;
      const int8_t* src = (m0 + m < M && k < kend) ? A + (size_t)(m0 + m) * K + k : zsrc;
      glds16_asm(src, slot + pc * 1024);
    } else if constexpr (BT) {
      const int q = pc - PA, n = 8 * q + (lane >> 3), c = (lane & 7) ^ ((n >> 1) & 7), k = k0 + 16 * c;
      const int8_t* src = (n < TN && n0 + n < N && k < kend) ? B + (size_t)(n0 + n) * K + k : zsrc;
      glds16_asm(src, slot + SA + q * 1024);
    } else {
      const int q = pc - PA, k = (1024 / TNP) * q + lane / CPR;
      const int b = (lane % CPR) ^ bswz<TNP>(k), n = n0 + 16 * b;
      const int8_t* src = (16 * b < TN && k0 + k < kend && n < N) ? B + (size_t)(k0 + k) * N + n : zsrc;
      glds16_asm(src, slot + SA + q * 1024);
    }
  };

#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v16i{0};
#pragma unroll
  for (int r = 0; r < PPW; ++r) issue_r(sb, r);
  const int q = (lane & 15) >> 1, p = lane & 1, g = (lane >> 4) & 1;
  for (int s = sb; s < se; ++s) {
    wait_vm0();  // this wave's pieces of stage s (stage s + 1 is issued below)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // the slot's fragment reads stay below the barrier
    const int8_t* la = lds + (s & 1) * SLOT;
    const int8_t* lb = la + SA;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      v4i fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = (wm * MI + i) * 32 + lr, c = ks * 2 + lh;
        fa[i] = *(const v4i*)(la + m * 128 + 16 * (c ^ ((m >> 1) & 7)));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (BT) {
          const int n = (wn * NJ + j) * 32 + lr, c = ks * 2 + lh;
          fb[j] = *(const v4i*)(lb + n * 128 + 16 * (c ^ ((n >> 1) & 7)));
        } else {
          const int k = ks * 32 + lh * 16 + q, b = (wn * NJ + j) * 2 + g;
          const int8_t* a0 = lb + k * TNP + 16 * (b ^ bswz<TNP>(k)) + 8 * p;
          const v2i lo = ds_tr8(a0), hi = ds_tr8(a0 + 8 * TNP);
          fb[j] = v4i{lo[0], lo[1], hi[0], hi[1]};
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
          // stage s + 1's pieces of this wave (into the slot stage s - 1
          // left), one after each of the stage's first PPW MFMAs: the matrix
          // pipe runs while they issue, instead of idling behind back-to-back
          // DMA issues after the barrier (the last stage issues a stage past
          // the range: zeros into a slot nobody reads, awaited after the loop)
          if ((ks * MI + i) * NJ + j < PPW) {
            __builtin_amdgcn_sched_barrier(0);
            issue_r(s + 1, (ks * MI + i) * NJ + j);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    }
  }
  wait_vm0();  // the past-range stage's pieces land before the LDS is reused or released
}

// acc -> C (int32 row-major), bounds-checked
template <int WN, int MI, int NJ>
__device__ __forceinline__ void k128_store(int32_t* __restrict__ C, int M, int N, int m0, int n0,
                                           const v16i (&acc)[MI][NJ]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 31, lh = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + (wn * NJ + j) * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M && n < N) C[(size_t)m * N + n] = acc[i][j][r];
      }
    }
}

template <int WM, int WN, int MI, int NJ, int WPS, bool BT = false>
__global__ __launch_bounds__(WM * WN * 64, WPS) void gemm_s8s8s32_k128_kernel(const int8_t* __restrict__ A,
                                                                             const int8_t* __restrict__ B,
                                                                             int32_t* __restrict__ C, int M, int N,
                                                                             int K, int nbn) {
  constexpr int NW = WM * WN, TM = 32 * WM * MI, TN = 32 * WN * NJ, TNP = b_pitch<TN>();
  static_assert(TNP == 256 || TNP == 128, "B image swizzle");
  constexpr int SA = TM * GK2, SLOT = SA + GK2 * TNP;
  constexpr int PA = TM / 8, PB = TNP / 8, NP = PA + PB, PPW = (NP + NW - 1) / NW;
  static_assert(PPW <= 4 * MI * NJ, "at most one piece per MFMA of a stage");
  static_assert(2 * SLOT <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * SLOT];
  // tile order: each XCD takes a contiguous run of l (xcd_remap), and l runs
  // down groups of GROW row blocks column by column, so the tiles an XCD's
  // CUs hold at once share GROW A panels and a few B panels in its L2
  constexpr int GROW = 4;
  const int l = xcd_remap(blockIdx.x, gridDim.x);
  const int nbm = (M + TM - 1) / TM, grp = l / (GROW * nbn), r0 = grp * GROW;
  const int gsz = nbm - r0 < GROW ? nbm - r0 : GROW, li = l - grp * GROW * nbn;
  const int m0 = (r0 + li % gsz) * TM, n0 = (li / gsz) * TN;
  v16i acc[MI][NJ];
  k128_tile<WM, WN, MI, NJ, BT>(A, B, M, N, K, m0, n0, 0, (K + GK2 - 1) / GK2, lds, acc);
  k128_store<WN, MI, NJ>(C, M, N, m0, n0, acc);
}

int num_cus_gemm() {
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

// Tile choice for the LDS-DMA kernel (knob "gemm_tile" forces one: 1 =
// 256 x 256, 2 = 256 x 128, 3 = 128 x 128).  tools/gemm_tiles.py, one box
// (TOPS for tiles 1 / 2 / 3): 8192^3 1878 / 1736 / 1515; 256 x 50176 x 2304
// 1491 / 1264 / 1118 and 50176 x 256 x 2304 1513 / 1298 / 1248 (the 256-wide
// side is read once: 256 x 256 wins although its 196 tiles leave CUs idle);
// 12544 x 512 x 4608 1009 / 1497 / 1374 (98 tiles of 256 x 256 idle 60 % of
// the chip); 128 x 200704 x 1152 655 / 585 / 775 (half of a 256-row tile
// would be padding).
// Tiles 4-6 have a 7-MFMA side (224): 256 x 224, 224 x 128, 224 x 256.
int gemm_tile_for(int M, int N) {
  const int forced = g_knob_gemm_tile.load(std::memory_order_relaxed);
  if (forced >= 1 && forced <= 6) return forced;
  if (M <= 128) return 3;
  const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
  if (t256 >= num_cus_gemm() || M <= 256 || N <= 256) return 1;
  return 2;
}

namespace {
template <bool BT>
hipError_t launch_gemm(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s) {
  // NN: K, N multiples of 16 (B rows are 16-byte chunks of N); NT: K alone
  const bool dma = K % 16 == 0 && (BT || N % 16 == 0) && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0;
  if (dma) {
    const int cfg = gemm_tile_for(M, N);
    static const int TMS[7] = {0, 256, 256, 128, 256, 224, 224}, TNS[7] = {0, 256, 128, 128, 224, 128, 256};
    const int TM = TMS[cfg], TN = TNS[cfg];
    const long tiles = (long)((M + TM - 1) / TM) * ((N + TN - 1) / TN);
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const int nbn = (N + TN - 1) / TN;
    if (cfg == 1)
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<2, 4, 4, 2, 1, BT>), dim3((unsigned)tiles), dim3(512), 0, s, A, B, C,
                         M, N, K, nbn);
    else if (cfg == 2)
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<4, 2, 2, 2, 1, BT>), dim3((unsigned)tiles), dim3(512), 0, s, A, B, C,
                         M, N, K, nbn);
    else if (cfg == 3)
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<2, 2, 2, 2, 2, BT>), dim3((unsigned)tiles), dim3(256), 0, s, A, B, C,
                         M, N, K, nbn);
    else if (cfg == 4)
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<8, 1, 1, 7, 1, BT>), dim3((unsigned)tiles), dim3(512), 0, s, A, B, C,
                         M, N, K, nbn);
    else if (cfg == 5)
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<1, 4, 7, 1, 1, BT>), dim3((unsigned)tiles), dim3(256), 0, s, A, B, C,
                         M, N, K, nbn);
    else
      hipLaunchKernelGGL((gemm_s8s8s32_k128_kernel<1, 8, 7, 1, 1, BT>), dim3((unsigned)tiles), dim3(512), 0, s, A, B, C,
                         M, N, K, nbn);
  } else {
    const int nbm = (M + GT - 1) / GT, nbn = (N + GT - 1) / GT;
    const long tiles = (long)nbm * nbn;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const int aligned = BT ? K % 16 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0
                           : K % 16 == 0 && N % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 7) == 0;
    hipLaunchKernelGGL(gemm_s8s8s32_generic_kernel<BT>, dim3((unsigned)tiles), dim3(512), 0, s, A, B, C, M, N, K, nbn,
                       aligned);
  }
  return hipGetLastError();
}
}  // namespace

hipError_t launch_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s) {
  return launch_gemm<false>(A, B, C, M, N, K, s);
}

// B supplied transposed: C[M][N] = A[M][K] . Bt[N][K]^T.
hipError_t launch_gemm_s8s8s32_nt(const int8_t* A, const int8_t* Bt, int32_t* C, int M, int N, int K, hipStream_t s) {
  return launch_gemm<true>(A, Bt, C, M, N, K, s);
}

}  // namespace dlq
