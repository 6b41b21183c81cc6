// Batched INT8 matmul with int8 output: the full contract surface of the
// reference's oneDNN wrapper dnnl_matmul_int8 (attention_cpu/dnnl_matmul_int8.cpp:7-75,
// declaration dnnl_matmul_int8.hpp:5-13).  The decoder itself never calls it
// (the weight GEMMs of gemm.hip keep fp32 outputs for the LayerNorm / residual
// path); it exists so that a caller of the reference's s8-output, BATCH form
// finds the same operation here.
//
//   A s8 [BATCH][M][K], B s8 [BATCH][K][N], C s8 [BATCH][M][N]   (format_tag abc, :20-27)
//   acc = sum_k A[b,m,k] * B[b,k,n]                                exact int32
//   y   = (float(acc) + bias[n]) * alpha,  alpha = scaleA * scaleB / scaleC   (:40-41)
//   y   = relu / gelu_erf (y)                                      (:43-50)
//   C   = round_half_even(saturate(y, -128, 127))
//
// The order (bias in the accumulator domain, then the output scale, then the
// post-op, then saturate-and-round) is oneDNN v2's reference matmul; oneDNN is
// absent from this image, so that order is restated, not pinned.
//
// Not a decode hot path: one 64 x 64 output tile per 256-thread workgroup,
// A and B tiles staged through LDS per 64-deep k-step (B transposed so each
// MFMA operand is one 16-byte LDS read), v_mfma_i32_16x16x64_i8.  Any M, N, K.
#include "common.hpp"

namespace llm {

namespace {

constexpr int kTile = 64;       // output rows / columns per workgroup
constexpr int kLdsStride = 80;  // bytes per staged row (64 + 16: 16-byte aligned)

__device__ __forceinline__ float s8_act(float y, int act) {
  if (act == LLM_ACT_RELU) return fmaxf(y, 0.f);
  if (act == LLM_ACT_GELU) return 0.5f * y * (1.f + erff(y * 0.70710678118654752f));
  return y;
}

__global__ __launch_bounds__(256) void i8_matmul_s8_kernel(const int8_t* __restrict__ A,
                                                           const int8_t* __restrict__ B,
                                                           int8_t* __restrict__ C, int M, int N,
                                                           int K, float alpha,
                                                           const float* __restrict__ bias,
                                                           int act) {
  __shared__ __attribute__((aligned(16))) uint8_t As[kTile * kLdsStride];
  __shared__ __attribute__((aligned(16))) uint8_t Bt[kTile * kLdsStride];  // [n][k]
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int n0 = blockIdx.x * kTile;
  const int m0 = blockIdx.y * kTile;
  const size_t b = blockIdx.z;
  const int8_t* Ab = A + b * (size_t)M * K;
  const int8_t* Bb = B + b * (size_t)K * N;

  i32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = i32x4{0, 0, 0, 0};

  const int ar = t >> 2, aq = (t & 3) * 16;  // A: row ar, k aq..aq+15 of the tile
  const int bk = t >> 2, bq = (t & 3) * 16;  // B: k bk, n bq..bq+15 of the tile
  for (int k0 = 0; k0 < K; k0 += kTile) {
    {
      const int m = m0 + ar;
      int8_t v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = k0 + aq + i;
        v[i] = (m < M && k < K) ? Ab[(size_t)m * K + k] : (int8_t)0;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) As[ar * kLdsStride + aq + i] = (uint8_t)v[i];
    }
    {
      const int k = k0 + bk;
      int8_t v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = n0 + bq + i;
        v[i] = (k < K && n < N) ? Bb[(size_t)k * N + n] : (int8_t)0;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) Bt[(bq + i) * kLdsStride + bk] = (uint8_t)v[i];
    }
    __syncthreads();
    // operands: lane l holds row (col) l & 15, k = 16 (l >> 4) .. + 15, the same
    // k order for A and B (gemm.hip), so the int32 dot product is exact
    const u32x4 af =
        *reinterpret_cast<const u32x4*>(As + (16 * w + (lane & 15)) * kLdsStride + 16 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x4 bf =
          *reinterpret_cast<const u32x4*>(Bt + (16 * j + (lane & 15)) * kLdsStride + 16 * (lane >> 4));
      acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, af),
                                                      __builtin_bit_cast(i32x4, bf), acc[j], 0, 0, 0);
    }
    __syncthreads();
  }

  // C/D layout: col = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma clang fp contract(off)
      const int m = m0 + 16 * w + 4 * (lane >> 4) + r;
      if (m >= M || n >= N) continue;
      float y = (float)acc[j][r];
      if (bias) y = y + bias[n];
      y = y * alpha;
      y = s8_act(y, act);
      y = fminf(fmaxf(y, -128.f), 127.f);
      C[b * (size_t)M * N + (size_t)m * N + n] = (int8_t)(int)__builtin_rintf(y);
    }
  }
}

}  // namespace

}  // namespace llm

using namespace llm;

extern "C" int i8_matmul_s8(const int8_t* A, const int8_t* B, int8_t* C, int batch, int M, int N,
                            int K, float scale_a, float scale_b, float scale_c, const float* bias,
                            int act, void* stream) {
  LLM_REQUIRE(batch >= 0 && M >= 0 && N >= 0 && K >= 0, "i8_matmul_s8: negative dimension");
  if ((size_t)batch * M * N == 0) return LLM_OK;
  LLM_REQUIRE(A && B && C, "i8_matmul_s8: NULL operand");
  LLM_REQUIRE(K < 131072, "i8_matmul_s8: K >= 131072 can overflow the int32 accumulator");
  LLM_REQUIRE(batch <= 65535 && (M + kTile - 1) / kTile <= 65535, "i8_matmul_s8: grid too large");
  LLM_REQUIRE(act >= LLM_ACT_NONE && act <= LLM_ACT_GELU, "i8_matmul_s8: bad activation");
  LLM_REQUIRE(scale_c != 0.f, "i8_matmul_s8: scale_c must be non-zero");
  const float alpha = scale_a * scale_b / scale_c;  // dnnl_matmul_int8.cpp:40
  const dim3 grid((unsigned)((N + kTile - 1) / kTile), (unsigned)((M + kTile - 1) / kTile),
                  (unsigned)batch);
  hipLaunchKernelGGL(i8_matmul_s8_kernel, grid, dim3(256), 0, as_stream(stream), A, B, C, M, N,
                     K, alpha, bias, act);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}
