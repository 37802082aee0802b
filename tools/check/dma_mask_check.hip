// dma_mask_check.hip -- test infrastructure, not product code: the masked
// LDS-DMA issues of the convs' shared piece plans (device_common.h
// glds16_asm_m / glds16_saddr_m) run for real (this file is compiled
// WITHOUT DLQ_PLAN_CAPTURE, which skips their asm).  One workgroup of two
// waves poisons a 4 KiB LDS region, then:
//   wave 0: glds16_asm_m   (valid = false) into [0, 1 KiB)   -- must not land
//           glds16_saddr_m (valid = false) into [1, 2 KiB)   -- must not land
//   wave 1: glds16_asm_m   (valid = true)  into [2, 3 KiB)   -- must land
//           glds16_saddr_m (valid = true)  into [3, 4 KiB)   -- must land
// each followed by a plain store from every lane (EXEC restored after the
// masked issue), then copies the region out.  An empty slot in the kernels
// re-issues another wave's piece (same bytes, same address), so the
// bit-exact network tests pass even if EXEC = 0 had no effect; this is the
// direct check (tests/test_gpu_dma_plan.py::test_masked_lds_dma).
// Linked into tools/check/libplancap.so (Makefile).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../dlq_amd/csrc/device_common.h"

namespace {
__global__ __launch_bounds__(128) void dma_mask_kernel(const int8_t* src, int8_t* out, int* lanes) {
  __shared__ __attribute__((aligned(16))) int8_t lds[4096];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  for (int i = t; i < 1024; i += 128) ((int*)lds)[i] = (int)0xa5a5a5a5;
  __syncthreads();
  const unsigned base = dlq::lds_addr32(lds);
  const bool valid = wave == 1;
  const int r = wave * 2;  // region of the asm form; r + 1: the saddr form
  dlq::glds16_asm_m(src + r * 1024 + lane * 16, base + r * 1024, valid);
  lanes[wave * 128 + lane] = lane + 1;  // every lane must store: EXEC restored
  dlq::glds16_saddr_m(src + (r + 1) * 1024, (unsigned)lane * 16, base + (r + 1) * 1024, valid);
  lanes[wave * 128 + 64 + lane] = lane + 1;
  dlq::wait_vm0();
  __syncthreads();
  for (int i = t; i < 1024; i += 128) ((int*)out)[i] = ((const int*)lds)[i];
}
}  // namespace

// src: 4096 device bytes, out: 4096, lanes: 256 ints.  Returns 0 or -1 (HIP error).
extern "C" int dmamask_run(const void* src, void* out, void* lanes) {
  hipLaunchKernelGGL(dma_mask_kernel, dim3(1), dim3(128), 0, 0, (const int8_t*)src, (int8_t*)out, (int*)lanes);
  return hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
