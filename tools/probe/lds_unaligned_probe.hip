// Probe (not product code): are 2-byte-aligned ds_read_b64 / ds_read_b128
// LDS reads exact on gfx950 under the runtime's default alignment mode, and
// what do they cost against aligned ones?  Each lane reads 8 (16) bytes at
// byte offset 2 * lane + shift (the stem's conv-column stride of 2 input
// pixels); the result is checked against the byte pattern, then a loop of
// 4096 reads per lane is timed with s_memtime (1 wave per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/lds_unaligned_probe.hip -o tools/probe/lds_unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int BYTES>
__global__ void rd(int shift, int stride, unsigned* bad, unsigned long long* cyc, unsigned* sink) {
  __shared__ unsigned char lds[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = (unsigned char)(i * 37 + (i >> 8));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned off = (unsigned)(stride * lane + shift);
  unsigned nbad = 0;
  if constexpr (BYTES == 8) {
    const unsigned long long v = *(const unsigned long long*)(lds + off);
    for (int b = 0; b < 8; ++b)
      if (((v >> (8 * b)) & 0xff) != (unsigned char)((off + b) * 37 + ((off + b) >> 8))) ++nbad;
  } else {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = *(const v4u*)(lds + off);
    for (int b = 0; b < 16; ++b)
      if (((v[b >> 2] >> (8 * (b & 3))) & 0xff) != (unsigned char)((off + b) * 37 + ((off + b) >> 8))) ++nbad;
  }
  atomicAdd(bad, nbad);
  unsigned acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 4096; ++it) {
    const unsigned o = (off + (it & 7) * 512) & 4095;
    if constexpr (BYTES == 8) {
      unsigned long long v;
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(o + (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds));
      acc += (unsigned)v ^ (unsigned)(v >> 32);
    } else {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      v4u v;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(o + (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds));
      acc += v[0] ^ v[3];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  unsigned *bad, *sink;
  unsigned long long* cyc;
  if (hipMalloc(&bad, 4) || hipMalloc(&sink, 1 << 20) || hipMalloc(&cyc, 8 * 1024)) return 3;
  const struct { int bytes, shift, stride; const char* what; } cases[] = {
      {8, 0, 8, "b64 aligned, stride 8"},   {8, 0, 2, "b64 stride 2 (even lanes aligned)"},
      {8, 2, 2, "b64 stride 2 shift 2"},    {8, 6, 2, "b64 stride 2 shift 6"},
      {16, 0, 16, "b128 aligned, stride 16"}, {16, 2, 2, "b128 stride 2 shift 2"},
      {8, 1, 2, "b64 odd byte offsets"}};
  for (auto& c : cases) {
    hipMemset(bad, 0, 4);
    if (c.bytes == 8)
      hipLaunchKernelGGL(rd<8>, dim3(1), dim3(64), 0, 0, c.shift, c.stride, bad, cyc, sink);
    else
      hipLaunchKernelGGL(rd<16>, dim3(1), dim3(64), 0, 0, c.shift, c.stride, bad, cyc, sink);
    if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", c.what); return 2; }
    unsigned hb;
    unsigned long long hc;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-36s wrong bytes %u   %.1f cycles per read (dependent, 1 wave)\n", c.what, hb, hc / 4096.0);
  }
  return 0;
}
