// Does v_mfma_f32_16x16x16_f16 keep small (normal) fp16 operands exactly?
// D = A . B with A[16][16] and B[16][16] fp16 from the host, lane maps
// A: row l&15, k 4(l>>4)+j; B: col l&15, k 4(l>>4)+j; D: col l&15, row 4(l>>4)+r.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x;
  f16x4 a, b;
  for (int j = 0; j < 4; ++j) {
    a[j] = A[(l & 15) * 16 + 4 * (l >> 4) + j];
    b[j] = B[(4 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f32x4 d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = d[r];
}
int main() {
  _Float16 hA[256], hB[256];
  float hD[256];
  srand(1);
  for (int i = 0; i < 256; ++i) hA[i] = (_Float16)((rand() % 2001 - 1000) / 1000.0f);
  for (int kk = 0; kk < 16; ++kk)
    for (int c = 0; c < 16; ++c) {
      float v = (rand() % 1000 + 1) / 1000.0f;              // col 0..3: ~0.5
      if (c >= 4 && c < 8) v *= 1e-3f;                      // col 4..7: ~5e-4 (normal)
      if (c >= 8 && c < 12) v *= 3e-5f;                     // col 8..11: subnormal range
      hB[kk * 16 + c] = (_Float16)v;
    }
  _Float16 *dA, *dB;
  float* dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  for (int c = 0; c < 16; c += 1) {
    double maxrel = 0, mag = 0;
    for (int r = 0; r < 16; ++r) {
      double s = 0;
      for (int kk = 0; kk < 16; ++kk) s += (double)(float)hA[r * 16 + kk] * (double)(float)hB[kk * 16 + c];
      maxrel = fmax(maxrel, fabs(hD[r * 16 + c] - s));
      mag = fmax(mag, fabs(s));
    }
    printf("col %2d  max |D - exact| %.3e  (|D| %.3e, rel %.3e)\n", c, maxrel, mag, maxrel / mag);
  }
  return 0;
}
