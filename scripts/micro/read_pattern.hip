// Microbenchmark: read-only HBM stream by access pattern and cache policy --
// is the 6.9 TB/s of read_stream (grid-stride float4) the ceiling for the
// attention scan's pattern (each wave streaming its own 8 KiB page pairs)?
//   pattern 0: grid-stride 1 KiB wave loads (read_stream)
//   pattern 1: each wave streams a contiguous run of RUN bytes, UNROLL 1 KiB
//              loads in flight (buffer_load_dwordx4, cache policy AUX)
//   pattern 2: as 1, but the wave's runs are 8 KiB pages at random places
// Prints TB/s per (pattern, aux, unroll, waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, int AUX, int PB = 8192>
__global__ __launch_bounds__(256) void run_kernel(const unsigned char* __restrict__ base,
                                                  const unsigned* __restrict__ page_of,
                                                  size_t pages_per_wave, unsigned* out) {
  constexpr int LPP = PB / 1024;  // wave loads per page
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  unsigned acc = 0;
  // UNROLL 1 KiB wave loads in flight
  const size_t nloads = pages_per_wave * LPP;
  for (size_t i0 = 0; i0 < nloads; i0 += UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t i = i0 + u;
      const size_t pg = page_of ? page_of[wave * pages_per_wave + (i / LPP)]
                                : wave * pages_per_wave + (i / LPP);
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(base + pg * PB), (short)0,
                                                        i < nloads ? PB : 0, 0x00020000);
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)((i % LPP) * 1024 + lane * 16), 0,
                                                   AUX);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) out[lane] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int U, int AUX, int PB = 8192>
int run(const unsigned char* p, const unsigned* pages, size_t waves, size_t ppw, unsigned* out,
        hipEvent_t a, hipEvent_t b, const char* name) {
  float best = 1e30f;
  const size_t threads = waves * 64;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((run_kernel<U, AUX, PB>), dim3((unsigned)(threads / 256)), dim3(256), 0, 0,
                       p, pages, ppw, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (rep > 0 && ms < best) best = ms;
  }
  const double bytes = (double)waves * ppw * PB;
  printf("%-8s aux %2d unroll %2d waves %6zu: %.3f TB/s (%.1f us)\n", name, AUX, U, waves,
         bytes / (best * 1e-3) / 1e12, best * 1e3);
  return 0;
}

int main() {
  const size_t bytes = 4ull << 30, npages = bytes / 8192;
  unsigned char* p; unsigned* out; unsigned* perm;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(p, 1, bytes));
  std::vector<unsigned> h(npages);
  for (size_t i = 0; i < npages; ++i) h[i] = (unsigned)i;
  srand(7);
  for (size_t i = npages - 1; i > 0; --i) { size_t j = (size_t)rand() % (i + 1); std::swap(h[i], h[j]); }
  CK(hipMalloc(&perm, npages * 4));
  CK(hipMemcpy(perm, h.data(), npages * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (size_t waves : {4096, 8192, 16384}) {
    const size_t ppw = npages / waves;
    run<8, 2>(p, nullptr, waves, ppw, out, a, b, "contig");
    run<8, 2>(p, perm, waves, ppw, out, a, b, "random");
    run<8, 0>(p, perm, waves, ppw, out, a, b, "random");
    run<8, 1>(p, perm, waves, ppw, out, a, b, "random");
    run<8, 3>(p, perm, waves, ppw, out, a, b, "random");
    run<8, 16>(p, perm, waves, ppw, out, a, b, "random");
    run<8, 18>(p, perm, waves, ppw, out, a, b, "random");
    run<16, 2>(p, perm, waves, ppw, out, a, b, "random");
    run<32, 2>(p, perm, waves, ppw, out, a, b, "random");
  }
  // C2's attention launch: 16 x 12 x 128 pages of 4 KiB (K 2 KiB + V 2 KiB),
  // 50 MB, as 768 / 1536 / 3072 waves (4 / 8 / 16 splits)
  for (size_t waves : {768, 1536, 3072}) {
    const size_t ppw = 24576 / waves;
    run<8, 2, 4096>(p, perm, waves, ppw, out, a, b, "c2-rand");
    run<16, 2, 4096>(p, perm, waves, ppw, out, a, b, "c2-rand");
    run<8, 2, 4096>(p, nullptr, waves, ppw, out, a, b, "c2-contig");
  }
  return 0;
}
