// stem.hip -- fused ResNet-18 stem: input quantisation + conv1 7x7/s2/p3 (+BN,
// ReLU, requant) + maxpool 3x3/s2/p1 in one kernel.
//
// Replaces (RK = CUDA/resnet18-kernel-lab/cpp/fp32): the input upload
// (RK/runtime/infer_e2e.cu:255-256), conv2d_nchw_im2col_gemm for conv1
// (:259-270, im2col_nchw + sgemm_tiled), bn_launch + relu_forward (:272-280)
// and maxpool2d_3x3_s2p1_nchw (:282-293).  The 112x112x64 conv1 output never
// leaves the register file.
//
// Input: every thread loads the fp32 values of its half super-pixel straight
// into registers (three 8-byte loads, one per channel: 64 lanes read 512
// contiguous bytes of an input row), PD steps ahead of their use, and
// quantises them into a ring of "super rows": 2x2 pixels x (RGB, 0) = 16-byte
// super-pixels, so the
// 7x7/s2 conv is a 4x4/s1 conv over super-pixels (kh = 2*ky+dy-1; kh = -1
// carries a zero weight) with K = 16 super taps x 16 B = 8 steps of
// v_mfma_i32_32x32x32_i8, every A fragment one ds_read_b128.
//
// MFMA orientation D[px][oc]: A = 32 conv pixels of one conv row, B = 32 output
// channels held in registers for the whole kernel.  A-row i is conv column
// c0 + pi(i) with pi chosen so that D register r of lane half h holds column
// c0 + 16h + r: each lane owns 16 consecutive columns of ONE channel, and the
// 3x3/s2 max pool runs on the int32 accumulators in registers (v_max3_i32).
// Pooling before the epilogue is exact because the epilogue y = fma(acc, a, b)
// -> clamp -> rne is monotone non-decreasing in acc once a >= 0; channels with
// a < 0 have their weights (and a) negated at packing time
// (dlq_pack_stem_weights_s8).  Only the pooled values (1/4 of the conv
// outputs) are requantised.
//
// Work item = (image, band of pooled rows).  8 waves = 2 channel tiles x 4
// column quarters; quarter q computes conv columns 28q-1 .. 28q+30 (32, of
// which 29 are used) and produces pooled columns 14q .. 14q+13.  A step
// computes conv rows 2p, 2p+1 and emits pooled row p.
#include <cmath>
#include <type_traits>
#include <utility>

#include "device_common.h"

namespace dlq {
namespace {

constexpr int SNW = 8;                   // waves
constexpr int PD = 2;                    // super-row pairs whose input loads are in flight ahead of the converter
constexpr int PATCH_SLOTS = 8;           // super-row ring
constexpr int PATCH_ROW = 128 * 16;      // super cols -4 .. 123
constexpr int OFF_PATCH = 0;
constexpr int OFF_STAGE = OFF_PATCH + PATCH_SLOTS * PATCH_ROW;  // per wave 16 x 32 B output staging
constexpr int WPITCH_S = 256 + 16;       // weight row pitch (17 units: a lane group's 16 rows on 16 bank quads)
constexpr int OFF_WST = OFF_STAGE + SNW * 512;                  // the 64 x 256 B weight image
constexpr int LDS_STEM = OFF_WST + 64 * WPITCH_S;               // 37 KiB: two workgroups per CU
static_assert(LDS_STEM <= 160 * 1024, "LDS budget");
constexpr int kIntMin = (int)0x80000000;

#ifdef DLQ_STAMPS
// timing-probe builds: per-wave cycle totals by section (no VM ops in the loop)
__device__ unsigned long long g_sstamps[512 * 8 * 8];
#define ST_DECL unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = __builtin_amdgcn_s_memtime()
#define ST(k)                                                       \
  do {                                                              \
    const unsigned long long st_now = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += st_now - st_prev;                                  \
    st_prev = st_now;                                               \
  } while (0)
#define ST_STORE()                                                                                       \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 512)                                                     \
      for (int q_ = 0; q_ < 6; ++q_) g_sstamps[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + q_] = st_acc[q_]; \
  } while (0)
#else
#define ST_DECL
#define ST(k) \
  do {        \
  } while (0)
#define ST_STORE() \
  do {             \
  } while (0)
#endif

struct StemArgs {
  const float* x;      // [N][3][224][224]
  const int8_t* w;     // [64][16 super taps][16 B] (dlq_pack_stem_weights_s8)
  const float* alpha;  // [64] |alpha| (packed), output-grid units
  const float* beta;   // [64]
  int8_t* y;           // [N][56][56][64]
  float inv_s;         // 1 / input scale
  int N, nb, R;        // batch, bands per image, pooled rows per band
};


__device__ __forceinline__ int max3i(int a, int b, int c) {
  return __builtin_elementwise_max(__builtin_elementwise_max(a, b), c);
}

// F8: the fp8 path: the input is quantised to e4m3 (enc4_f8),
// the 8 i8 k-steps become 4 v_mfma_f32_32x32x64_f8f6f4 (k-steps 2i, 2i+1 as
// the two halves of each 32-byte fragment, A and B alike), the pool runs on
// the fp32 accumulators (max is exact; the e4m3 epilogue is monotone once
// alpha >= 0: dlq_pack_stem_weights_f8 flips the sign bits of the rows with
// alpha < 0).
template <bool F8>
__global__ __launch_bounds__(SNW * 64, 4) void stem_fused_kernel(StemArgs a) {
  using Acc = typename std::conditional<F8, v16f, v16i>::type;
  using Pv = typename std::conditional<F8, float, int>::type;
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_STEM];
  const unsigned lds32 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int ot = wave & 1, q = wave >> 1;  // channel tile, column quarter
  const int nitems = a.N * a.nb;

  // The weight image in LDS (B fragments re-read per conv row: registers go to
  // the second co-resident workgroup), and the channel's epilogue constants.
  for (int i = tid; i < 64 * 16; i += SNW * 64)
    *(v4i*)(lds + OFF_WST + (i >> 4) * WPITCH_S + (i & 15) * 16) = *(const v4i*)(a.w + i * 16);
  const int8_t* wlds = lds + OFF_WST + (ot * 32 + lr) * WPITCH_S + lh * 16;
  const float al = a.alpha[ot * 32 + lr], be = a.beta[ot * 32 + lr];
  __syncthreads();
  // A-row permutation: lane row i -> conv column offset pi(i) (D reg r of half h = column 16h + r)
  const int pi = ((lr >> 3) << 2) + (lr & 3) + 16 * ((lr >> 2) & 1);
  const int a_unit = 28 * q + 1 + pi;  // super-col unit of tap kx = 0 (unit = super col + 4)
  int8_t* stg = lds + OFF_STAGE + wave * 512;

  ST_DECL;
  for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
    const int n = item / a.nb, band = item - n * a.nb;
    const int py0 = band * a.R, py1 = min(56, py0 + a.R);
    if (py0 >= py1) continue;
    const int sr0 = 2 * py0 - 3;  // first super row (pair k = super rows sr0+2k, sr0+2k+1)
    const float* img = a.x + (size_t)n * 3 * 224 * 224;

    // Super-row pair k = super rows sr0+2k, sr0+2k+1.  Thread = (pixel row
    // dy, super row h of the pair, unit): unit = super col + 4 (units 0..3
    // and 116..127 are the zero border); its input = channels 0..2 x pixels
    // (2 sc, 2 sc + 1) of image row 2 sr + dy: three float2 loads.  Pair k's
    // loads sit in register set k % (PD + 1) (compile-time: the step loop is
    // unrolled by PD + 1) until convert_pair quantises them into the patch.
    const int cv_unit = tid & 127, cv_h = (tid >> 7) & 1, cv_dy = tid >> 8, cv_sc = cv_unit - 4;
    using F2 = float __attribute__((ext_vector_type(2)));
    F2 raw[PD + 1][3];
    auto load_pair = [&](int k, F2 (&r)[3]) {
      const int sr = sr0 + 2 * k + cv_h;
      if ((unsigned)sr < 112u && (unsigned)cv_sc < 112u) {
        const float* src = img + (size_t)(2 * sr + cv_dy) * 224 + 2 * cv_sc;
#pragma unroll
        for (int c = 0; c < 3; ++c) r[c] = *(const F2*)(src + (size_t)c * 224 * 224);
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) r[c] = F2{0.f, 0.f};
      }
    };
    // Quantise pair k into two super rows of the patch ring: each thread
    // writes the 8 bytes of its dy (dx = 0, 1) of one super-pixel.
    auto convert_pair = [&](int k, const F2 (&r)[3]) {
      const int sr = sr0 + 2 * k + cv_h;
      int2 out = {0, 0};
      if ((unsigned)sr < 112u && (unsigned)cv_sc < 112u) {
        if constexpr (F8) {  // (c0, c1, c2, +0) e4m3 per pixel
          out.x = (int)enc4_f8(r[0][0] * a.inv_s, r[1][0] * a.inv_s, r[2][0] * a.inv_s, 0.f, -448.f);
          out.y = (int)enc4_f8(r[0][1] * a.inv_s, r[1][1] * a.inv_s, r[2][1] * a.inv_s, 0.f, -448.f);
        } else {
          unsigned u[3][2];  // [c][dx]: clamp(x/s) + 1.5*2^23 -> rne'd int8 in the low byte
#pragma unroll
          for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx)
              u[c][dx] = __float_as_uint(__builtin_amdgcn_fmed3f(r[c][dx] * a.inv_s, -127.f, 127.f) + 12582912.0f);
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {  // bytes (c0, c1, c2, 0)
            const unsigned t = __builtin_amdgcn_perm(u[1][dx], u[0][dx], 0x0c0c0400u);
            (dx ? out.y : out.x) = (int)__builtin_amdgcn_perm(u[2][dx], t, 0x0c040100u);
          }
        }
      }
      *(int2*)(lds + OFF_PATCH + (sr & (PATCH_SLOTS - 1)) * PATCH_ROW + cv_unit * 16 + cv_dy * 8) = out;
    };
    // One conv row (global row oy): the wave's 32 px x 32 oc tile, 8 k-steps.
    // int8: fragments stream two k-steps ahead through a 3-deep ring of
    // untracked ds_read_b128 (inline asm: the compiler can neither hoist all
    // 16 reads nor keep them all live -- two workgroups share the registers).
    const unsigned a_col = lds32 + OFF_PATCH + (a_unit + lh) * 16;
    const unsigned w_row = lds32 + (unsigned)(wlds - lds);
    auto conv_row = [&](int oy) {
      Acc acc = Acc{0};
      unsigned ra[4];  // super rows oy-2 .. oy+1 (ky = 0..3)
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) ra[ky] = a_col + ((oy - 2 + ky) & (PATCH_SLOTS - 1)) * PATCH_ROW;
      if constexpr (F8) {  // k-steps 2kp, 2kp+1 = the two halves of one 64-deep fp8 MFMA
        v4i fa[2][2], fw[2][2];
#define STEM_RD8(kp)                                                                                              \
  asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(fa[(kp) & 1][0]) : "v"(ra[kp]) : "memory");                   \
  asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(fa[(kp) & 1][1]) : "v"(ra[kp]) : "memory");                  \
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fw[(kp) & 1][0]) : "v"(w_row), "n"(64 * (kp)) : "memory");  \
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fw[(kp) & 1][1]) : "v"(w_row), "n"(64 * (kp) + 32) : "memory")
#define STEM_K8(kp)                                                                                               \
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(fa[(kp) & 1][0]), "+v"(fa[(kp) & 1][1]), "+v"(fw[(kp) & 1][0]),        \
               "+v"(fw[(kp) & 1][1]) : "n"((kp) + 1 < 4 ? 4 : 0) : "memory");                                     \
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(cat8(fa[(kp) & 1][0], fa[(kp) & 1][1]),                       \
                                                        cat8(fw[(kp) & 1][0], fw[(kp) & 1][1]), acc, 0, 0, 0, 0, 0, 0)
        STEM_RD8(0);
        STEM_RD8(1);
        STEM_K8(0);
        STEM_RD8(2);
        STEM_K8(1);
        STEM_RD8(3);
        STEM_K8(2);
        STEM_K8(3);
#undef STEM_RD8
#undef STEM_K8
      } else {
        v4i fa[3], fw[3];
#define STEM_RD(kk)                                                                                    \
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[(kk) % 3]) : "v"(ra[(kk) >> 1]), "n"(32 * ((kk) & 1)) \
               : "memory");                                                                          \
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fw[(kk) % 3]) : "v"(w_row), "n"(32 * (kk)) : "memory")
#define STEM_K(kk)                                                                                     \
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(fa[(kk) % 3]), "+v"(fw[(kk) % 3]) : "n"((kk) + 1 < 8 ? 2 : 0)    \
               : "memory");                                                                          \
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[(kk) % 3], fw[(kk) % 3], acc, 0, 0, 0)
        STEM_RD(0);
        STEM_RD(1);
        STEM_K(0);
        STEM_RD(2);
        STEM_K(1);
        STEM_RD(3);
        STEM_K(2);
        STEM_RD(4);
        STEM_K(3);
        STEM_RD(5);
        STEM_K(4);
        STEM_RD(6);
        STEM_K(5);
        STEM_RD(7);
        STEM_K(6);
        STEM_K(7);
#undef STEM_RD
#undef STEM_K
      }
      return acc;
    };
    auto mx3 = [](Pv x, Pv y, Pv z) -> Pv {
      if constexpr (F8)
        return __builtin_fmaxf(__builtin_fmaxf(x, y), z);
      else
        return max3i(x, y, z);
    };
    const Pv kLow = F8 ? (Pv)-INFINITY : (Pv)kIntMin;
    // Horizontal 3-max of a conv row, H[m] = max(local cols 2m, 2m+1, 2m+2):
    // half 0 takes column 16 from half 1; quarter 0's column 0 is conv column
    // -1 (pool padding).  Half 1's H[6], H[7] and half 0's beyond m=7 are unused.
    auto hpool = [&](Acc c, Pv (&H)[8]) {
      unsigned x0 = __builtin_bit_cast(unsigned, c[0]), c16 = x0;
      swap32(x0, c16);  // lanes 0-31: c16 = lanes 32-63's c[0]
      const Pv c0v = (q == 0 && lh == 0) ? kLow : c[0];
      H[0] = mx3(c0v, c[1], c[2]);
#pragma unroll
      for (int m = 1; m < 7; ++m) H[m] = mx3(c[2 * m], c[2 * m + 1], c[2 * m + 2]);
      H[7] = mx3(c[14], c[15], __builtin_bit_cast(Pv, c16));
    };

    // ---- prologue: pairs 0..2 converted (super rows 2py0-3 .. 2py0+2),
    // pairs 3 .. 2+PD loaded; H of conv row 2py0-1.
    static_assert(PD == 2, "prologue ring assignment below assumes 3 register sets");
    load_pair(0, raw[0]);
    load_pair(1, raw[1]);
    load_pair(2, raw[2]);
    convert_pair(0, raw[0]);
    load_pair(3, raw[0]);
    convert_pair(1, raw[1]);
    load_pair(4, raw[1]);
    convert_pair(2, raw[2]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): patch rows written (loads stay in flight)
    __builtin_amdgcn_s_barrier();
    Pv Hp[8];
    if (py0 == 0) {
#pragma unroll
      for (int m = 0; m < 8; ++m) Hp[m] = kLow;  // conv row -1: pool padding
    } else {
      hpool(conv_row(2 * py0 - 1), Hp);
    }

    // The staged output of step p is read back and stored during step p+1
    // (after its convert), so the LDS round trip and the store issue overlap
    // the next step instead of closing this one.
    const int pxl = lane >> 1, hf = lane & 1;
    auto store_row = [&](int p) {
      const v4i o = *(const v4i*)(stg + pxl * 32 + hf * 16);
      if (lane < 28) *(v4i*)(a.y + (((size_t)n * 56 + p) * 56 + 14 * q + pxl) * 64 + ot * 32 + hf * 16) = o;
    };
    // step t (pooled row p = py0 + t): pair t+3 (register set (t+3) % 3 =
    // t % 3) is quantised for the next step, pair t+5 is loaded into the set
    // pair t+2 freed, conv rows 2p and 2p+1 are computed and pooled.
    auto step = [&](int t, auto setc) {
      constexpr int S = decltype(setc)::value;  // == t % 3
      const int p = py0 + t;
      ST(5);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): last step's patch rows and staging
      __builtin_amdgcn_s_barrier();
      ST(0);
      convert_pair(t + 3, raw[S]);
      ST(1);
      if (t > 0) store_row(p - 1);
      load_pair(t + 5, raw[(S + 2) % 3]);
      ST(2);

      Pv He[8], Ho[8];
      hpool(conv_row(2 * p), He);
      hpool(conv_row(2 * p + 1), Ho);
      ST(3);
      // vertical max, epilogue on the pooled values, bytes -> staging [16 px][32 oc]
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const Pv v = mx3(Hp[m], He[m], Ho[m]);
        Hp[m] = Ho[m];
        const float y = __builtin_fmaf((float)v, al, be);
        if constexpr (F8) {
          stg[(m + 8 * lh) * 32 + lr] = (int8_t)enc4_f8(y, 0.f, 0.f, 0.f, 0.f);
        } else {
          const unsigned u = __float_as_uint(__builtin_amdgcn_fmed3f(y, 0.f, 127.f) + 12582912.0f);
          stg[(m + 8 * lh) * 32 + lr] = (int8_t)u;
        }
      }
      // 14 pooled columns x 32 channels = 28 x 16 B, staged in LDS (written by
      // this wave: LDS is in order); stored during the next step
      ST(4);
    };
    const int nsteps = py1 - py0;
    int t = 0;
    for (; t + 3 <= nsteps; t += 3) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
      step(t + 2, std::integral_constant<int, 2>{});
    }
    if (t < nsteps) step(t, std::integral_constant<int, 0>{});
    if (t + 1 < nsteps) step(t + 1, std::integral_constant<int, 1>{});
    if (py1 > py0) store_row(py1 - 1);
    wait_vm0();
    __syncthreads();  // ring reuse by the next item
  }
  ST_STORE();
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

// OIHW int8 q[64][3][7][7] -> [64][ky 4][kx 4][dy 2][dx 2][c 4] with
// kh = 2ky+dy-1, kw = 2kx+dx-1; rows of channels with alpha < 0 are negated
// and |alpha| returned, which keeps the fused stem's pool-before-epilogue exact.
void pack_stem_weights(const int8_t* q, const float* alpha, int8_t* out, float* alpha_abs) {
  for (int i = 0; i < 64 * 256; ++i) out[i] = 0;
  for (int o = 0; o < 64; ++o) {
    const bool neg = alpha[o] < 0.f;
    alpha_abs[o] = neg ? -alpha[o] : alpha[o];
    for (int ky = 0; ky < 4; ++ky)
      for (int kx = 0; kx < 4; ++kx)
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx) {
            const int kh = 2 * ky + dy - 1, kw = 2 * kx + dx - 1;
            if (kh < 0 || kw < 0) continue;
            for (int c = 0; c < 3; ++c) {
              const int v = q[((o * 3 + c) * 7 + kh) * 7 + kw];
              out[o * 256 + (((ky * 4 + kx) * 2 + dy) * 2 + dx) * 4 + c] = (int8_t)(neg ? -v : v);
            }
          }
  }
}

// e4m3 twin: the sign bit is the negation.
void pack_stem_weights_f8(const uint8_t* q, const float* alpha, uint8_t* out, float* alpha_abs) {
  for (int i = 0; i < 64 * 256; ++i) out[i] = 0;
  for (int o = 0; o < 64; ++o) {
    const bool neg = alpha[o] < 0.f;
    alpha_abs[o] = neg ? -alpha[o] : alpha[o];
    for (int ky = 0; ky < 4; ++ky)
      for (int kx = 0; kx < 4; ++kx)
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx) {
            const int kh = 2 * ky + dy - 1, kw = 2 * kx + dx - 1;
            if (kh < 0 || kw < 0) continue;
            for (int c = 0; c < 3; ++c) {
              const uint8_t v = q[((o * 3 + c) * 7 + kh) * 7 + kw];
              out[o * 256 + (((ky * 4 + kx) * 2 + dy) * 2 + dx) * 4 + c] = neg ? (uint8_t)(v ^ 0x80) : v;
            }
          }
  }
}

hipError_t launch_stem_fused(const float* x, int N, const int8_t* w, const float* alpha, const float* beta,
                             float inv_s, int8_t* y, hipStream_t s, bool f8) {
  const int ncu = num_cus_stem();
  int nb = (2 * ncu + N - 1) / N;  // bands per image so that every CU gets two co-resident items
  nb = nb < 1 ? 1 : (nb > 14 ? 14 : nb);
  const int R = (56 + nb - 1) / nb;
  nb = (56 + R - 1) / R;
  StemArgs a{x, w, alpha, beta, y, inv_s, N, nb, R};
  const int items = N * nb, grid = items < 2 * ncu ? items : 2 * ncu;
  if (f8)
    hipLaunchKernelGGL(stem_fused_kernel<true>, dim3(grid), dim3(SNW * 64), 0, s, a);
  else
    hipLaunchKernelGGL(stem_fused_kernel<false>, dim3(grid), dim3(SNW * 64), 0, s, a);
  return hipGetLastError();
}

}  // namespace dlq
