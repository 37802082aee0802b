// gemm.hip -- dlq_gemm_s8s8s32: C[M][N] (int32) = A[M][K] . B[K][N] (int8),
// row-major, any M, N, K: the int8 replacement of the reference's exported
// sgemm_tiled (RK/kernels/sgemm_tiled.cu:5-46, called by
// conv2d_nchw_im2col_gemm RK/runtime/infer_e2e.cu:129-133 with A = OIHW
// weights [OC][IC*kH*kW], B = im2col [IC*kH*kW][OH*OW]).  int32 sums are
// exact, so any k order gives the reference's accumulators bit for bit.
//
// Tile 256 x 256 per 512-thread workgroup (8 waves = 2 (M) x 4 (N), each 128 x
// 64 = 4 x 2 v_mfma_i32_32x32x32_i8 tiles), K = 64 per stage, double-buffered
// LDS (2 x 40 KiB), one barrier per stage: the next stage's global loads are
// in flight in registers while this stage's MFMAs run.
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

__global__ __launch_bounds__(512, 1) void gemm_s8s8s32_kernel(const int8_t* __restrict__ A,
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
  v4i ra[2];
  unsigned rb[4][2];

  auto gload = [&](int k0) {
    if (full_mn && k0 + GK <= K) {
#pragma unroll
      for (int p = 0; p < 2; ++p) ra[p] = *(const v4i*)(A + (size_t)(m0 + a_row + 128 * p) * K + k0 + a_ch * 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint2 v = *(const uint2*)(B + (size_t)(k0 + 4 * b_rq + r) * N + n0 + 8 * b_cg);
        rb[r][0] = v.x;
        rb[r][1] = v.y;
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int m = m0 + a_row + 128 * p, k = k0 + a_ch * 16;
      const int8_t* src = A + (size_t)m * K + k;
#pragma unroll
      for (int w = 0; w < 4; ++w) ra[p][w] = (int)(m < M ? ld_bytes(src + 4 * w, K - k - 4 * w) : 0u);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 4 * b_rq + r, n = n0 + 8 * b_cg;
      const int8_t* src = B + (size_t)k * N + n;
      rb[r][0] = k < K ? ld_bytes(src, N - n) : 0u;
      rb[r][1] = k < K ? ld_bytes(src + 4, N - n - 4) : 0u;
    }
  };
  auto lstore = [&](int slot) {
    int8_t* la = lds + slot * GSLOT;
    int8_t* lb = la + GT * GP;
#pragma unroll
    for (int p = 0; p < 2; ++p) *(v4i*)(la + (a_row + 128 * p) * GP + a_ch * 16) = ra[p];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // 4 x 4 byte transpose: rows k..k+3 -> column dwords
      const unsigned t0 = __builtin_amdgcn_perm(rb[1][h], rb[0][h], 0x05010400u);
      const unsigned t1 = __builtin_amdgcn_perm(rb[1][h], rb[0][h], 0x07030602u);
      const unsigned t2 = __builtin_amdgcn_perm(rb[3][h], rb[2][h], 0x05010400u);
      const unsigned t3 = __builtin_amdgcn_perm(rb[3][h], rb[2][h], 0x07030602u);
      const unsigned d[4] = {__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
                             __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u)};
#pragma unroll
      for (int c = 0; c < 4; ++c) *(unsigned*)(lb + (8 * b_cg + 4 * h + c) * GP + 4 * b_rq) = d[c];
    }
  };

  v16i acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = v16i{0};
  const int nst = (K + GK - 1) / GK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    if (s + 1 < nst) gload((s + 1) * GK);
    const int8_t* la = lds + (s & 1) * GSLOT;
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
    if (s + 1 < nst) lstore((s + 1) & 1);
    __syncthreads();
  }
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

}  // namespace

hipError_t launch_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s) {
  const int nbm = (M + GT - 1) / GT, nbn = (N + GT - 1) / GT;
  const long tiles = (long)nbm * nbn;
  if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
  const int aligned = K % 16 == 0 && N % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 7) == 0;
  hipLaunchKernelGGL(gemm_s8s8s32_kernel, dim3((unsigned)tiles), dim3(512), 0, s, A, B, C, M, N, K, nbn, aligned);
  return hipGetLastError();
}

}  // namespace dlq
