// One-wave-per-row LayerNorm (+ int8 quantisation) of the weight GEMM's
// LayerNorm prologue (gemm.hip), plus the quantise / fp16 helpers the
// LayerNorm launch (row_ops.hip layernorm_rows_kernel, 256 threads per row)
// shares with it.
//
// LayerNorm<T>::forward (decoder/layer_norm.hpp:20-37): biased variance,
// inv_std = 1.0 / sqrt(var + eps) (double division of the float sqrt), y =
// ((x - mean) * inv_std) * gamma + beta, every step rounded (no contraction);
// int8_quant.cpp:5-13,59-64: scale = 127 / (absmax + 1e-6), q = clamp(round(y *
// scale), -128, 127), dequantisation factor 1 / scale.
//
// Row layout per lane: float4 chunks c = 64 j + lane (j < CPL), i.e. lane l
// holds elements 4 (64 j + l) .. +3 — every load instruction of the wave reads
// 1 KiB contiguous (fully coalesced), and every output is one dword (4 int8)
// or 8 bytes (4 fp16) per chunk.  The reduction order does not depend on the
// output type, and any CPL that covers the row gives the same bits (empty
// chunks add exact zeros).
#pragma once

#include "common.hpp"

namespace llm {

// Wave-wide max with DPP row moves (every lane ends with the maximum).
__device__ __forceinline__ float ln_wave_max(float x) {
  x = fmaxf(x, mov_dpp<0xB1>(x));   // quad_perm [1,0,3,2]
  x = fmaxf(x, mov_dpp<0x4E>(x));   // quad_perm [2,3,0,1]
  x = fmaxf(x, mov_dpp<0x141>(x));  // row_half_mirror
  x = fmaxf(x, mov_dpp<0x140>(x));  // row_mirror
  x = fmaxf(x, __shfl_xor(x, 16, 64));
  return fmaxf(x, __shfl_xor(x, 32, 64));
}

template <int CPL>
struct LnRow {
  f32x4 v[CPL];
};

// Issue the loads of one row of K4 float4 chunks (!ok: zeros).
template <int CPL>
__device__ __forceinline__ void ln_wave_load(const float* __restrict__ row, int K4, bool ok,
                                             LnRow<CPL>& r) {
  const int lane = lane_id();
  const f32x4* row4 = reinterpret_cast<const f32x4*>(row);
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = 64 * j + lane;
    r.v[j] = (ok && c < K4) ? row4[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// The same chunks from an fp16 row (an embedding row: TokenEmbedding::forward,
// decoder/token_embedding.hpp:19-26, widened exactly).
template <int CPL>
__device__ __forceinline__ void ln_wave_load_f16(const _Float16* __restrict__ row, int K4, bool ok,
                                                 LnRow<CPL>& r) {
  const int lane = lane_id();
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4* row4 = reinterpret_cast<const h4*>(row);
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = 64 * j + lane;
    const h4 h = (ok && c < K4) ? row4[c] : h4{0, 0, 0, 0};
    r.v[j] = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
}

// Embedding row of token id tok (clamped to [0, V), as embed_kernel).
__device__ __forceinline__ const _Float16* ln_embed_row(const _Float16* E, const int32_t* tok,
                                                        int m, int V, int K) {
  int t = tok[m];
  t = t < 0 ? 0 : (t >= V ? V - 1 : t);
  return E + (size_t)t * K;
}

// x -> LN(x) in place; returns the row's |max| (wave-uniform).
template <int CPL>
__device__ __forceinline__ float ln_wave_compute(LnRow<CPL>& x, const LnRow<CPL>& gm,
                                                 const LnRow<CPL>& bt, int K, float eps) {
  const int lane = lane_id();
  const int K4 = K >> 2;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) s += (x.v[j][0] + x.v[j][1]) + (x.v[j][2] + x.v[j][3]);
  const float mean = group_sum<64>(s) / (float)K;
  float vs = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    if (64 * j + lane >= K4) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = x.v[j][e] - mean;
      vs = fmaf(d, d, vs);
    }
  }
  const float var = group_sum<64>(vs) / (float)K;
  const float inv_std = (float)(1.0 / (double)sqrtf(var + eps));
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float y = __fmul_rn(__fmul_rn(x.v[j][e] - mean, inv_std), gm.v[j][e]);
      x.v[j][e] = __fadd_rn(y, bt.v[j][e]);
      am = fmaxf(am, fabsf(x.v[j][e]));  // empty chunks: beta 0 -> 0
    }
  return ln_wave_max(am);
}

// 4 values -> 4 int8 in one dword (int8_quant.cpp quantize_to_int8 semantics)
__device__ __forceinline__ uint32_t ln_quant4(f32x4 y, float scale) {
  uint32_t wd = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float t = roundf(__fmul_rn(y[e], scale));
    t = fminf(fmaxf(t, -128.f), 127.f);
    wd |= (uint32_t)(uint8_t)(int8_t)(int)t << (8 * e);
  }
  return wd;
}

typedef _Float16 ln_f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ ln_f16x4 ln_half4(f32x4 y) {
  return ln_f16x4{(_Float16)y[0], (_Float16)y[1], (_Float16)y[2], (_Float16)y[3]};
}

}  // namespace llm
