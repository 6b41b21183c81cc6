// Where a stream's workgroups land: each workgroup of census_kernel records
// its XCC id and HW_ID (CU / SH / SE) -- used to map the bits of
// hipExtStreamCreateWithCUMask onto XCDs (scripts/overlap_probe.py).
// Built as a shared library: hipcc --offload-arch=gfx950 -shared -fPIC.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void census_kernel(uint32_t* out, int spin) {
  uint32_t hw = 0, xcc = 0;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // keep the workgroup resident a while so the grid spreads over every CU it may use
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < spin) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

extern "C" int census(uint32_t* out_dev, int blocks, int spin, void* stream) {
  hipLaunchKernelGGL(census_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out_dev, spin);
  return (int)hipGetLastError();
}
