// Microbenchmark: every workgroup reads the SAME buffer of S bytes (the
// activation rows a fused GEMM prologue reads), coalesced float4 loads,
// 8 waves per workgroup; vs each workgroup reading its own S bytes.
// Prints per-launch time and per-CU rate.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(512) void rd(const f4* __restrict__ p, size_t n4, size_t wg_stride4,
                                          float* out) {
  const f4* q = p + blockIdx.x * wg_stride4;
  float s = 0.f;
  for (size_t i = threadIdx.x; i < n4; i += 512 * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * 512 < n4 ? q[i + u * 512] : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u][0] + v[u][1] + v[u][2] + v[u][3];
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
int main() {
  float* buf; float* out;
  CK(hipMalloc(&buf, 256 << 20)); CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 0, 256 << 20));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (size_t S : {48u << 10, 256u << 10, 512u << 10}) {
    for (int own = 0; own < 2; ++own) {
      for (int grid : {192, 256}) {
        const size_t n4 = S / 16;
        float best = 1e9;
        for (int r = 0; r < 8; ++r) {
          CK(hipEventRecord(a));
          hipLaunchKernelGGL(rd<8>, dim3(grid), dim3(512), 0, 0, (const f4*)buf, n4, own ? n4 : 0, out);
          CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
          float ms; CK(hipEventElapsedTime(&ms, a, b)); if (r > 0 && ms < best) best = ms;
        }
        printf("S %4zu KB %s grid %d: %7.2f us  (%.0f GB/s per WG)\n", S >> 10, own ? "own " : "same", grid,
               best * 1e3, S / (best * 1e-3) / 1e9);
      }
    }
  }
  return 0;
}
