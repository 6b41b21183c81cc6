// Microbenchmark: read-only HBM stream ceiling on MI355X (what the paged
// attention scan is bounded by).  Each lane loads 16 B per access, UNROLL
// independent loads in flight, grid-stride over a 4 GiB buffer; the sum is
// written once per wave so nothing is optimised away.  Prints TB/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ p, size_t n16,
                                                   unsigned* out) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  for (size_t i = tid; i < n16; i += stride * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = i + (size_t)u * stride;
      if (NT) v[u] = j < n16 ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
      else v[u] = j < n16 ? p[j] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) out[tid & 1023] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int U, bool NT>
int run(const u32x4* p, size_t n16, unsigned* out, int grid, hipEvent_t a, hipEvent_t b) {
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((read_kernel<U, NT>), dim3(grid), dim3(256), 0, 0, p, n16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (rep > 0 && ms < best) best = ms;
  }
  printf("unroll %2d nt %d grid %6d: %.3f TB/s (%.1f us)\n", U, NT, grid,
         n16 * 16.0 / (best * 1e-3) / 1e12, best * 1e3);
  return 0;
}

int main() {
  const size_t bytes = 4ull << 30, n16 = bytes / 16;
  u32x4* p; unsigned* out;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(p, 1, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int grid : {2048, 4096, 8192, 16384}) {
    run<4, true>(p, n16, out, grid, a, b);
    run<8, true>(p, n16, out, grid, a, b);
    run<8, false>(p, n16, out, grid, a, b);
    run<16, true>(p, n16, out, grid, a, b);
  }
  return 0;
}
