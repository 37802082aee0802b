// device_common.h -- device-side types and helpers shared by the gfx950 kernels.
#pragma once
#include <type_traits>

#include "dlq_internal.h"

namespace dlq {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef signed char v16c __attribute__((ext_vector_type(16)));

constexpr int BK = 64;   // K bytes per pipeline step = two 32-deep MFMA k-steps
constexpr int NT = 256;  // threads per conv workgroup (4 waves)

// 16-byte chunk swizzle inside a 64-byte LDS row: lanes of one ds_read_b128
// group read 16 different rows at the same chunk; XOR with (row>>2)&3 spreads
// them over all 64 banks (MI355X_MICROARCH.md §LDS lane groups).
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// clamp(rne(y), +-127) -- the requantisation of the int8 scheme.
__device__ __forceinline__ int sat_rne(float y) {
  float q = __builtin_rintf(y);
  q = q < -127.f ? -127.f : q;
  q = q > 127.f ? 127.f : q;
  return (int)q;
}

// Fused-epilogue requantisation of 4 values already in output-grid units:
// q = rne(clamp(y, lo, 127)) packed as 4 x int8.  clamp = one v_med3_f32;
// adding 1.5*2^23 rounds to nearest-even and leaves q in the low mantissa
// bits (two's complement in the low byte for |q| <= 127); two v_perm_b32 + or
// pack the bytes.  Bit-identical to oracle.c ora_epilogue_s8's
// rintf(clamp(y)).
__device__ __forceinline__ unsigned quant4(float y0, float y1, float y2, float y3, float lo) {
  const float M = 12582912.0f;
  const unsigned u0 = __float_as_uint(__builtin_amdgcn_fmed3f(y0, lo, 127.f) + M);
  const unsigned u1 = __float_as_uint(__builtin_amdgcn_fmed3f(y1, lo, 127.f) + M);
  const unsigned u2 = __float_as_uint(__builtin_amdgcn_fmed3f(y2, lo, 127.f) + M);
  const unsigned u3 = __float_as_uint(__builtin_amdgcn_fmed3f(y3, lo, 127.f) + M);
  return __builtin_amdgcn_perm(u1, u0, 0x0c0c0400u) | __builtin_amdgcn_perm(u3, u2, 0x04000c0cu);
}

typedef float v2f __attribute__((ext_vector_type(2)));

// Fused epilogue of 4 accumulators (one MFMA-layout register group):
// y = fma(float(acc), alpha, beta) [+ fma(float(res byte), r_s, y)], then
// quant4 -- scalar FMAs, bit-identical to oracle.c.  The kernel files that
// use them are compiled with -fno-slp-vectorize (Makefile): packed
// v_pk_fma_f32 forms cost more beside the partner wave's MFMAs
// (MI355X_MICROARCH.md, 'price of one filler'); measured on the network:
// stride-2 family 35.1 -> 34.3 us per launch, logits bit-identical
// (profiles/r05_ab_episc.txt).
__device__ __forceinline__ unsigned epi4(const int* acc, const float* al, const float* be, float lo) {
  return quant4(__builtin_fmaf((float)acc[0], al[0], be[0]), __builtin_fmaf((float)acc[1], al[1], be[1]),
                __builtin_fmaf((float)acc[2], al[2], be[2]), __builtin_fmaf((float)acc[3], al[3], be[3]), lo);
}
__device__ __forceinline__ unsigned epi4_res(const int* acc, const float* al, const float* be, unsigned r4, float r_s,
                                             float lo) {
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    y[e] = __builtin_fmaf((float)(int)(signed char)(r4 >> (8 * e)), r_s, __builtin_fmaf((float)acc[e], al[e], be[e]));
  return quant4(y[0], y[1], y[2], y[3], lo);
}

// ReLU requantisation without the med3 / magic-number / perm sequence:
// rne(clamp(y, 0, 127)) = v_cvt_pk_u8_f32(min(y, 127)), which rounds to
// nearest even, saturates at 0 and inserts the byte in one instruction
// (equal on every fp32 pattern of [-2, 300] and a stride of the whole finite
// range: tools/probe/cvt_pk_u8_probe.hip).  Byte e = value e, as quant4.
__device__ __forceinline__ unsigned quant4_relu(float y0, float y1, float y2, float y3) {
  unsigned r = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(y0, 127.f), 0, 0u);
  r = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(y1, 127.f), 1, r);
  r = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(y2, 127.f), 2, r);
  return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(y3, 127.f), 3, r);
}
__device__ __forceinline__ unsigned epi4_relu(const int* acc, const float* al, const float* be) {
  return quant4_relu(__builtin_fmaf((float)acc[0], al[0], be[0]), __builtin_fmaf((float)acc[1], al[1], be[1]),
                     __builtin_fmaf((float)acc[2], al[2], be[2]), __builtin_fmaf((float)acc[3], al[3], be[3]));
}
__device__ __forceinline__ unsigned epi4_res_relu(const int* acc, const float* al, const float* be, unsigned r4,
                                                  float r_s) {
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    y[e] = __builtin_fmaf((float)(int)(signed char)(r4 >> (8 * e)), r_s, __builtin_fmaf((float)acc[e], al[e], be[e]));
  return quant4_relu(y[0], y[1], y[2], y[3]);
}

// The downsample residual computed in place (conv3x3i.hip DSR): the 1x1/s2
// downsample's accumulators `accd` requantised exactly as its own epilogue
// would store them (rd = rne(clamp(fma(accd, ald, bed), -127, 127)), the int8
// value held as a float: v_med3_f32 + v_rndne_f32), then used as conv2's
// residual: y = fma(rd, r_s, fma(acc, al, be)) -> ReLU requantisation.
// Bit-identical to storing rd as int8 and reading it back (epi4_res_relu).
__device__ __forceinline__ unsigned epi4_dsr_relu(const int* acc, const float* al, const float* be, const int* accd,
                                                  const float* ald, const float* bed, float r_s) {
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float rd = __builtin_rintf(__builtin_amdgcn_fmed3f(__builtin_fmaf((float)accd[e], ald[e], bed[e]), -127.f, 127.f));
    y[e] = __builtin_fmaf(rd, r_s, __builtin_fmaf((float)acc[e], al[e], be[e]));
  }
  return quant4_relu(y[0], y[1], y[2], y[3]);
}

// ---- fp8 (e4m3, OCP) helpers: DESIGN.md §3b, oracle.c ora_*_f8 ----------
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v8i cat8(v4i lo, v4i hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); }

// requant of 4 values to e4m3: clamp(y, lo, 448) (v_med3), -0 -> +0 (+0.0f),
// round-to-nearest-even encode (v_cvt_pk_fp8_f32, byte j = value j).
// Bit-identical to oracle.c f8_requant (tests/test_gpu_f8.py).
__device__ __forceinline__ unsigned enc4_f8(float y0, float y1, float y2, float y3, float lo) {
  const float c0 = __builtin_amdgcn_fmed3f(y0, lo, 448.f) + 0.0f;
  const float c1 = __builtin_amdgcn_fmed3f(y1, lo, 448.f) + 0.0f;
  const float c2 = __builtin_amdgcn_fmed3f(y2, lo, 448.f) + 0.0f;
  const float c3 = __builtin_amdgcn_fmed3f(y3, lo, 448.f) + 0.0f;
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(c0, c1, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c2, c3, r, true);
  return (unsigned)r;
}

// e4m3 twins of epi4 / epi4_res on fp32 accumulators (packed fmas, then
// enc4_f8): per element the same IEEE sequence as the generic fp8 kernel.
__device__ __forceinline__ unsigned epi4_f8(const float* acc, const float* al, const float* be, float lo) {
  const v2f y01 = __builtin_elementwise_fma(v2f{acc[0], acc[1]}, v2f{al[0], al[1]}, v2f{be[0], be[1]});
  const v2f y23 = __builtin_elementwise_fma(v2f{acc[2], acc[3]}, v2f{al[2], al[3]}, v2f{be[2], be[3]});
  return enc4_f8(y01[0], y01[1], y23[0], y23[1], lo);
}
__device__ __forceinline__ unsigned epi4_res_f8(const float* acc, const float* al, const float* be, unsigned r4,
                                                float r_s, float lo) {
  const v2f s = {r_s, r_s};
  v2f y01 = __builtin_elementwise_fma(v2f{acc[0], acc[1]}, v2f{al[0], al[1]}, v2f{be[0], be[1]});
  v2f y23 = __builtin_elementwise_fma(v2f{acc[2], acc[3]}, v2f{al[2], al[3]}, v2f{be[2], be[3]});
  y01 = __builtin_elementwise_fma(
      v2f{__builtin_amdgcn_cvt_f32_fp8((int)r4, 0), __builtin_amdgcn_cvt_f32_fp8((int)r4, 1)}, s, y01);
  y23 = __builtin_elementwise_fma(
      v2f{__builtin_amdgcn_cvt_f32_fp8((int)r4, 2), __builtin_amdgcn_cvt_f32_fp8((int)r4, 3)}, s, y23);
  return enc4_f8(y01[0], y01[1], y23[0], y23[1], lo);
}

// Bijective XCD-aware remap: consecutive logical tiles land on one XCD
// (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Work split of a launch's n_items over its blocks: logical block b =
// xcd_remap(blockIdx.x) takes items b, b + gridDim, ... (count of them).
// (Contiguous ranges of a balanced partition instead, so that XCD x works on
// the same eighth of the batch in every layer, were measured and removed: no
// gain on the wide convs, the stride-2 convs 1.5-2 us slower per launch,
// tools/ab.py on one box)
__device__ __forceinline__ void xcd_chunk(int n_items, int& first, int& count) {
  const int Gd = gridDim.x, b = xcd_remap(blockIdx.x, Gd);
  first = b;
  count = n_items > b ? (n_items - b + Gd - 1) / Gd : 0;
}
// item index of the block's li-th item under xcd_chunk
__device__ __forceinline__ int xcd_item(int first, int li) {
  return first + li * (int)gridDim.x;
}

// One 16-byte LDS-DMA per lane: global (per-lane address) -> LDS at the
// wave-uniform `lds_wave_base` + 16*lane (global_load_lds_dwordx4).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One LDS-DMA piece (1 KiB: 16 B per lane to lds_addr + 16*lane) issued from
// asm.  The builtin carries an LDS memory operand, which hipcc's waitcnt pass
// treats as a possible FLAT-LDS access: every later ds_read wait then becomes
// lgkmcnt(0), draining the fragment prefetch.  Completion must be covered by
// the caller's explicit vmcnt counts + barrier.
#ifdef DLQ_PLAN_CAPTURE
// Plan-capture builds (tools/check/plan_capture.hip, never libdlq.so): every
// LDS-DMA piece is recorded instead of issued -- its M0 LDS address and the
// 64 lanes' source addresses, in issue order per (workgroup, wave) -- so the
// host checker (tools/check/dma_plan.py) is compared with the compiled
// kernels' own plans (tests/test_gpu_dma_plan.py).
struct PlanPiece {
  unsigned long long src[64];
  unsigned lds, pad[3];
};
__device__ PlanPiece* g_cap_buf;
__device__ unsigned* g_cap_cnt;
__device__ unsigned g_cap_max;
__device__ unsigned g_cap_nw;    // waves the host sized g_cap_cnt / g_cap_buf for
__device__ unsigned g_cap_drop;  // pieces not recorded (wave or record index out of range)
__device__ __forceinline__ void plan_capture(const void* gsrc, unsigned lds_addr) {
  const int lane = threadIdx.x & 63;
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w >= g_cap_nw) {  // a grid larger than the host's buffers: count, never write past them
    if (lane == 0) atomicAdd(&g_cap_drop, 1u);
    return;
  }
  unsigned i = 0;
  if (lane == 0) i = atomicAdd(&g_cap_cnt[w], 1u);
  i = (unsigned)__shfl((int)i, 0);
  if (i >= g_cap_max && lane == 0) atomicAdd(&g_cap_drop, 1u);
  if (i < g_cap_max) {
    PlanPiece* r = g_cap_buf + (size_t)w * g_cap_max + i;
    r->src[lane] = (unsigned long long)(uintptr_t)gsrc;
    if (lane == 0) r->lds = lds_addr;
  }
}
#endif

__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_addr) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
#ifdef DLQ_PLAN_CAPTURE
  plan_capture(gsrc, m0);
  return;
#endif
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "{m0}"(m0) : "memory");
}

// One LDS-DMA piece whose 64 sources are a wave-uniform base + a per-lane
// 32-bit offset (the saddr form: base in an SGPR pair, computed by the
// compiler in 64-bit pointer arithmetic from uniform values).
__device__ __forceinline__ void glds16_saddr(const void* base, unsigned voff, unsigned lds_addr) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
#ifdef DLQ_PLAN_CAPTURE
  plan_capture((const char*)base + voff, m0);
  return;
#endif
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base), "{m0}"(m0) : "memory");
}

// Predicated twins of glds16_asm / glds16_saddr for piece plans whose kind
// at each issue slot is the same for every wave (one code path for all waves
// of a workgroup): a wave with no piece at this slot issues the instruction
// with EXEC = 0 (no lane reads or writes anything; `gsrc` / `base` must
// still be an address the wave could read).  No branch is involved, so the
// surrounding MFMA / LDS schedule (sched_group_barrier) stays one block.  Every
// counted wait in the kernels covers only VM ops YOUNGER than the awaited one
// (stores, residual loads), so whether the hardware counts a masked piece in
// vmcnt cannot change what those waits guarantee.  EXEC is SET to the mask
// (the ballot of `valid`: all active lanes or none), never AND-ed: an
// s_and_b64 writes SCC, which the compiler may hold live across the asm (it
// faulted an s_cselect-chosen address on the GPU); s_mov_b64 leaves SCC.
__device__ __forceinline__ void glds16_asm_m(const void* gsrc, unsigned lds_addr, bool valid) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
#ifdef DLQ_PLAN_CAPTURE
  if (valid) plan_capture(gsrc, m0);
  return;
#endif
  const unsigned long long mask = __builtin_amdgcn_ballot_w64(valid);  // an SGPR pair: all lanes or none
  unsigned long long saved;
  asm volatile(
      "s_mov_b64 %0, exec\n\ts_mov_b64 exec, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(saved)
      : "v"(gsrc), "{m0}"(m0), "s"(mask)
      : "memory");
}
__device__ __forceinline__ void glds16_saddr_m(const void* base, unsigned voff, unsigned lds_addr, bool valid) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
#ifdef DLQ_PLAN_CAPTURE
  if (valid) plan_capture((const char*)base + voff, m0);
  return;
#endif
  const unsigned long long mask = __builtin_amdgcn_ballot_w64(valid);  // an SGPR pair: all lanes or none
  unsigned long long saved;
  asm volatile(
      "s_mov_b64 %0, exec\n\ts_mov_b64 exec, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(saved)
      : "v"(voff), "s"(base), "{m0}"(m0), "s"(mask)
      : "memory");
}

// The next launch's weight regions (ConvArgs::pf) pulled towards the CUs:
// one 1 KiB LDS-DMA piece per wave of the grid (pieces numbered across both
// regions, spread over every wave), landing in an LDS area nobody reads (an
// idle ring slot), so no VGPR is written behind the compiler's back.  The
// launch's own counted waits see these as older VM ops: issue them where
// every later wait may cover them (a last stage, no DMA after).
__device__ __forceinline__ void prefetch_next(const Prefetch& pf, int wave, int nw, unsigned lds_dummy) {
  const int lane = threadIdx.x & 63;
  int q = blockIdx.x * nw + wave;
  const int G = gridDim.x * nw;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!pf.p[r]) continue;
    const int per = pf.len[r] >> 10, tot = pf.n[r] * per;
    for (; q < tot; q += G) {
      const int blk = q / per, off = (q - blk * per) * 1024;
      glds16_asm((const int8_t*)pf.p[r] + (size_t)blk * pf.stride[r] + off + lane * 16, lds_dummy);
    }
    q -= tot;
  }
}

// LDS byte address of a __shared__ pointer (for M0).
__device__ __forceinline__ unsigned lds_addr32(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// v_permlane32_swap_b32: lanes 32-63 of x <-> lanes 0-31 of y.
__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

// 16-byte global load the compiler does not track: its completion is awaited
// only by an explicit counted wait, so hipcc's waitcnt pass cannot turn a
// loop-carried load into a vmcnt(0) drain of an LDS-DMA ring.
__device__ __forceinline__ v4i gload16_untracked(const void* p) {
  v4i r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

typedef int v2i __attribute__((ext_vector_type(2)));

// ds_read_b64_tr_b8: per 16-lane group, lane 2q + p addresses row q (of 8),
// bytes 8p .. 8p+7; lane i receives column i's 8 row bytes, byte q = row q.
__device__ __forceinline__ v2i ds_tr8(const int8_t* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)p);
}

// MFMA-layout <-> store-layout exchange for a 32x32 int8 output tile (see
// conv3x3w.hip): q[g] holds channels 8g + 4h .. +3 of this lane's pixel (h =
// lane half); afterwards {q0, q2, q1, q3} are channels 16h .. 16h+15.
__device__ __forceinline__ v4i mfma_to_store16(unsigned q0, unsigned q1, unsigned q2, unsigned q3) {
  swap32(q0, q2);
  swap32(q1, q3);
  return v4i{(int)q0, (int)q2, (int)q1, (int)q3};
}

// s_waitcnt vmcnt(N) expcnt(7) lgkmcnt(0) for a wave-uniform runtime N <= 63
// (gfx9 encoding: vmcnt[3:0] in bits 3:0, vmcnt[5:4] in bits 15:14).  A
// builtin per case so hipcc's waitcnt pass sees every wait.
template <int N>
__device__ __forceinline__ void wait_vm_const() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}
template <int N>
__device__ __forceinline__ void wait_vm_sel(int n) {
  if constexpr (N < 63) {
    if (n == N) { wait_vm_const<N>(); return; }
    wait_vm_sel<N + 1>(n);
  } else {
    wait_vm_const<63>();
  }
}
__device__ __forceinline__ void wait_vm(int n) { wait_vm_sel<0>(n); }

// The LDS input patch of a stride-1, pad-1 3x3 conv over a tile of
// consecutive output pixels [p0, pend) (NHWC, pixel p = (n*H + oh)*W + ow):
// the tile's rows plus a one-row halo above and below each image it touches,
// no halo columns (taps left/right of the image read a zero region instead).
// Slot order: image n0's rows oh0-1 .. (cnt0 slots), then each further image's
// rows -1 .. H (H+2 slots each); a patch pixel index is slot*W + column.
struct PatchTile {
  int p0, pend, n0, oh0, cnt0, slots;
};

__device__ __forceinline__ PatchTile patch_tile(int p0, int pend, int W, int H) {
  PatchTile t;
  t.p0 = p0;
  t.pend = pend;
  const int R0 = p0 / W, R1 = (pend - 1) / W;
  t.n0 = R0 / H;
  t.oh0 = R0 - t.n0 * H;
  const int n1 = R1 / H;
  t.cnt0 = ((n1 == t.n0) ? (R1 - R0) : (H - 1 - t.oh0)) + 3;
  t.slots = (n1 == t.n0) ? t.cnt0 : t.cnt0 + (n1 - t.n0 - 1) * (H + 2) + (R1 - n1 * H) + 3;
  return t;
}

// slot -> (image, input row); the row may be -1 or H (halo outside the image).
__device__ __forceinline__ void patch_slot(const PatchTile& t, int slot, int H, int& n, int& ih) {
  if (slot < t.cnt0) {
    n = t.n0;
    ih = t.oh0 - 1 + slot;
  } else {
    const int s2 = slot - t.cnt0;
    n = t.n0 + 1 + s2 / (H + 2);
    ih = s2 % (H + 2) - 1;
  }
}

// Output pixel p of the tile -> patch pixel index of its tap (kh=0, kw=1)
// (= the pixel directly above), and the 9-bit mask of taps inside the image.
__device__ __forceinline__ void patch_pixel(const PatchTile& t, int p, int W, int H, int& base, unsigned& mask) {
  base = 0;
  mask = 0;
  if (p >= t.pend) return;
  const int n = p / (H * W), r = p - n * (H * W), oh = r / W, ow = r - oh * W;
  const int slot0 = (n == t.n0) ? oh - t.oh0 : t.cnt0 + (n - t.n0 - 1) * (H + 2) + oh;
  base = slot0 * W + ow;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      if ((unsigned)(oh + kh - 1) < (unsigned)H && (unsigned)(ow + kw - 1) < (unsigned)W) mask |= 1u << (kh * 3 + kw);
}

}  // namespace dlq
