// device_common.h -- device-side types and helpers shared by the gfx950 kernels.
#pragma once
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

// Bijective XCD-aware remap: consecutive logical tiles land on one XCD
// (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// One 16-byte LDS-DMA per lane: global (per-lane address) -> LDS at the
// wave-uniform `lds_wave_base` + 16*lane (global_load_lds_dwordx4).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace dlq
