// Microbenchmark: per-kernel cost of a chain of dependent launches captured in
// one hipGraph (the decode step's structure), vs the kernel's grid size and
// vs a trivial body.  Prints us per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void touch_kernel(float* x, int n) {  // one read + write per thread
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 1.0001f + 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* d; float* x;
  CK(hipMalloc(&d, 64));
  CK(hipMalloc(&x, 64 << 20));
  CK(hipMemset(d, 0, 64));
  CK(hipMemset(x, 0, 64 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int N = 200;
  struct Cfg { const char* name; int grid, block, kind; } cfgs[] = {
    {"empty 1x64", 1, 64, 0}, {"empty 64x256", 64, 256, 0}, {"empty 256x256", 256, 256, 0},
    {"empty 1024x256", 1024, 256, 0}, {"empty 256x1024", 256, 1024, 0},
    {"touch 64x256 (16K floats)", 64, 256, 1}, {"touch 512x256 (128K floats)", 512, 256, 1},
  };
  for (auto& c : cfgs) {
    for (int graph = 0; graph < 2; ++graph) {
      hipGraphExec_t ge = nullptr;
      auto enqueue = [&]() {
        for (int i = 0; i < N; ++i) {
          if (c.kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(c.grid), dim3(c.block), 0, st, d);
          else hipLaunchKernelGGL(touch_kernel, dim3(c.grid), dim3(c.block), 0, st, x, c.grid * c.block);
        }
      };
      if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        enqueue();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      float best = 1e30f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a, st));
        if (graph) CK(hipGraphLaunch(ge, st)); else enqueue();
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("%-30s %-6s %7.2f us/kernel\n", c.name, graph ? "graph" : "eager", best * 1000.f / N);
      if (ge) CK(hipGraphExecDestroy(ge));
    }
  }
  return 0;
}
