// Shared host/device helpers for the gfx950 decode path.
#pragma once

#ifndef LLM_TUNING
#define LLM_TUNING 0  // 1: the tuning library (Makefile `tune`)
#endif

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "llm_decoder.h"

namespace llm {

// Integer tuning knob from the environment (dflt when unset or empty).
inline int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// Thread-local last-error message (llm_last_error()).
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);

#define LLM_HIP_RET(expr)                                                        \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess)                                                        \
      return ::llm::fail(LLM_ERR_HIP, std::string(#expr " failed: ") +           \
                                          hipGetErrorString(_e));                \
  } while (0)

#define LLM_REQUIRE(cond, msg)                                                   \
  do {                                                                           \
    if (!(cond)) return ::llm::fail(LLM_ERR_INVALID, msg);                       \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr float kNegSentinel = -1.0e30f;  // "minus infinity" that stays finite
constexpr float kLog2e = 1.4426950408889634f;

// Counted fixed-point accumulator of the FP16 decoder's fused o_proj
// (pa_decode.hip, workgroup merge): the H (row, head) workgroups of a row each
// add their head's product o_h . W_o[h] into one int64 per output column as
// 2^56 (an arrival count in the top bits) + the product in units of 2^-32.
// Integer addition is order-independent, so the sum is the same bits whatever
// order the heads' atomics land in (fp32 atomics would not be), and the adder
// whose returned old value counts H - 1 arrivals holds the complete sum: it
// stores the fp32 value and clears the column for the next layer.  Exact to
// 2^-33 per head for |sum| < 2^23 (8.4e6) and H <= 64.
//
// Range guard: the count bits stay intact only while |sum| < 2^23.  Each
// head's term is therefore clamped to |v| <= oacc_limit(H) = (2^23 - 1) / H,
// so H terms can never reach 2^23, and a NaN maps to the positive limit.  A
// clamped term sets *flag (a plain vector store; the decoder turns it into
// LLM_ERR_RANGE at llm_decoder_sync / the next synchronous step).  The
// column then still completes after exactly H arrivals and is cleared, so an
// out-of-range value costs that one output, never the later layers or steps.
constexpr float kOAccScale = 4294967296.f;  // 2^32
constexpr long long kOAccCount = 1LL << 56;
__host__ __device__ __forceinline__ float oacc_limit(int H) {
  return (float)((1 << 23) - 1) / (float)H;
}
__device__ __forceinline__ long long oacc_term(float v, float lim, bool& clamped) {
  const bool ok = fabsf(v) <= lim;  // false for NaN and +-inf
  clamped = !ok;
  const float c = ok ? v : (v < 0.f ? -lim : lim);
  return __float2ll_rn(c * kOAccScale) + kOAccCount;
}
__device__ __forceinline__ int oacc_count(long long v) {
  return (int)((v + (kOAccCount >> 1)) >> 56);
}
__device__ __forceinline__ float oacc_value(long long v) {
  const long long f = v - (long long)oacc_count(v) * kOAccCount;
  return (float)((double)f * (1.0 / 4294967296.0));
}

// DPP lane moves (row = 16 lanes).  ctrl must be a compile-time constant.
template <int CTRL>
__device__ __forceinline__ float mov_dpp(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}

// Sum over aligned groups of G lanes (G in {2,4,8,16,32,64}); every lane of a
// group ends with the identical total (commutative butterfly).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
  if constexpr (G >= 2) x += mov_dpp<0xB1>(x);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) x += mov_dpp<0x4E>(x);   // quad_perm [2,3,0,1]
  if constexpr (G >= 8) x += mov_dpp<0x141>(x);  // row_half_mirror
  if constexpr (G >= 16) x += mov_dpp<0x140>(x); // row_mirror
  if constexpr (G >= 32) x += __shfl_xor(x, 16, 64);
  if constexpr (G >= 64) x += __shfl_xor(x, 32, 64);
  return x;
}

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = fmaxf(x, __shfl_xor(x, off, 64));
  return x;
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ int wave_id_uniform() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Offset of activation element (m, k) in MFMA A-fragment order ("packed A"):
// one contiguous 1 KiB block per (16-row tile, k-step), lane l of the block
// holding row l&15 and 16 B of k (16 int8 or 8 fp16) — the exact operand
// layout of v_mfma_i32_16x16x64_i8 / v_mfma_f32_16x16x32_f16, so the GEMM
// reads each fragment with one coalesced buffer_load_dwordx4.
// KS = k-steps per row (K/64 for int8, K/32 for fp16).  Offsets in elements.
__host__ __device__ __forceinline__ size_t a_frag_off_i8(int m, int k, int KS) {
  return ((size_t)((m >> 4) * KS + (k >> 6)) * 64 + (m & 15) + 16 * ((k & 63) >> 4)) * 16 + (k & 15);
}
__host__ __device__ __forceinline__ size_t a_frag_off_f16(int m, int k, int KS) {
  return ((size_t)((m >> 4) * KS + (k >> 5)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
}

}  // namespace llm
