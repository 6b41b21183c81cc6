// Decode-shaped weight GEMMs on gfx950 MFMA.
//
//   i8_gemm : v_mfma_i32_16x16x64_i8, exact int32 accumulate, fp32 epilogue
//             (qkv_proj / o_proj / mlp_fc1 / mlp_fc2 of INT8Decoder; contract of
//             dnnl_matmul_int8, attention_cpu/dnnl_matmul_int8.cpp:7-75)
//   f16_gemm: v_mfma_f32_16x16x32_f16 (CUDADecoder weights; MLP<T>::forward,
//             decoder/mlp.hpp:23-41)
//   lm_head : x . E^T with x split into fp16 hi + lo (two MFMAs per step)
//
// Decode GEMMs have M = rows in flight (<= 64 per block) and stream every
// weight byte once: they are HBM-bound (128 op/B at M = 64 vs a ~625 op/B
// ridge).  So the design is a weight stream, not a compute tile:
//   * weights are repacked once at load time into MFMA B-fragment order:
//     for every (16-column tile, k-step) one contiguous 1 KiB block in which
//     lane l's 16 bytes are exactly its B operand -> one fully coalesced
//     buffer_load_dwordx4 per MFMA;
//   * a 512-thread workgroup owns one 16-column tile x up to 64 rows and its
//     8 waves split K; each wave issues 4 k-steps of loads before its MFMAs
//     (all of a decode GEMM's weight bytes are in flight at once), partial
//     accumulators are summed through LDS in a fixed order (deterministic),
//     then the fused dequant / bias / activation epilogue writes fp32.
//   * the k order inside a fragment (lane group l>>4 holds k = 16*(l>>4)+j) is
//     the same for A and B, so the dot product is exact whatever the
//     hardware's internal k permutation; C/D layout: col = lane&15,
//     row = 4*(lane>>4) + reg (cdna_hip_programming.md §3).
#include "common.hpp"

namespace llm {

struct GemmArgs {
  const uint8_t* A;
  int lda;            // elements
  const uint8_t* B;   // packed weights, or E rows for the LM head
  int M, N, K, KS;    // KS = number of k-steps
  const float* sa;
  const float* sw;
  const float* bias;
  int act;
  float* C;
  int32_t* acc_out;
};

constexpr int kGemmWaves = 8;
constexpr int kUnroll = 4;

__device__ __forceinline__ float apply_act(float y, int act) {
  if (act == LLM_ACT_RELU) return fmaxf(y, 0.f);
  if (act == LLM_ACT_GELU) return 0.5f * y * (1.f + erff(y * 0.70710678118654752f));
  return y;
}

enum class GemmKind { I8, F16, LMHEAD };

template <GemmKind KIND>
struct GemmTraits;
template <>
struct GemmTraits<GemmKind::I8> {
  static constexpr int KSTEP = 64, ESIZE = 1;
  using acc_t = i32x4;
};
template <>
struct GemmTraits<GemmKind::F16> {
  static constexpr int KSTEP = 32, ESIZE = 2;
  using acc_t = f32x4;
};
template <>
struct GemmTraits<GemmKind::LMHEAD> {
  static constexpr int KSTEP = 32, ESIZE = 4;  // A is fp32
  using acc_t = f32x4;
};

template <GemmKind KIND, int MT>
__global__ __launch_bounds__(512) void gemm_kernel(GemmArgs a) {
  using Tr = GemmTraits<KIND>;
  using acc_t = typename Tr::acc_t;
  constexpr int KSTEP = Tr::KSTEP;
  __shared__ __attribute__((aligned(16))) acc_t red[kGemmWaves][MT][64];

  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int ntile = blockIdx.x;
  const int m0 = blockIdx.y * 16 * MT;
  const int ks0 = (w * a.KS) / kGemmWaves;
  const int ks1 = ((w + 1) * a.KS) / kGemmWaves;

  // A descriptor: rows >= M (and anything past the matrix) read as zero.
  const uint32_t a_bytes = (uint32_t)((size_t)a.M * a.lda * Tr::ESIZE);
  const auto arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a_bytes, 0x00020000);
  // B descriptor
  uint32_t b_bytes;
  const uint8_t* bbase;
  if constexpr (KIND == GemmKind::LMHEAD) {
    bbase = a.B;  // E [N][K] fp16
    b_bytes = (uint32_t)((size_t)a.N * a.K * 2);
  } else {
    bbase = a.B + (size_t)ntile * a.KS * 1024;
    b_bytes = (uint32_t)a.KS * 1024u;
  }
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, (short)0, b_bytes, 0x00020000);

  const int arow_lane = lane & 15;
  const int kgrp = lane >> 4;
  uint32_t a_row_off[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = m0 + mt * 16 + arow_lane;
    a_row_off[mt] = row < a.M ? (uint32_t)((size_t)row * a.lda * Tr::ESIZE) : 0xFFFFFFF0u;
  }
  uint32_t b_lane_off;
  if constexpr (KIND == GemmKind::LMHEAD) {
    const int n = ntile * 16 + arow_lane;
    b_lane_off = n < a.N ? (uint32_t)((size_t)n * a.K * 2) + kgrp * 16 : 0xFFFFFFF0u;
  } else {
    b_lane_off = lane * 16;
  }

  acc_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = acc_t{0, 0, 0, 0};

  for (int ks = ks0; ks < ks1; ks += kUnroll) {
    u32x4 bf[kUnroll];
    u32x4 af[kUnroll][MT];
    u32x4 af2[kUnroll][MT];  // LMHEAD: second 16 bytes of the fp32 A fragment
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const bool ok = ks + u < ks1;
      const int kk = ks + u;
      uint32_t boff;
      if constexpr (KIND == GemmKind::LMHEAD)
        boff = ok ? b_lane_off + (uint32_t)kk * KSTEP * 2 : 0xFFFFFFF0u;
      else
        boff = ok ? (uint32_t)kk * 1024u + b_lane_off : 0xFFFFFFF0u;
      bf[u] = __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff, 0, 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint32_t koff = (uint32_t)(kk * KSTEP + kgrp * (KSTEP / 4)) * Tr::ESIZE;
        const uint32_t aoff = (ok && a_row_off[mt] != 0xFFFFFFF0u) ? a_row_off[mt] + koff : 0xFFFFFFF0u;
        af[u][mt] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, aoff, 0, 0);
        if constexpr (KIND == GemmKind::LMHEAD)
          af2[u][mt] = __builtin_amdgcn_raw_buffer_load_b128(
              arsrc, aoff == 0xFFFFFFF0u ? aoff : aoff + 16, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if constexpr (KIND == GemmKind::I8) {
          acc[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, af[u][mt]),
                                                          __builtin_bit_cast(i32x4, bf[u]),
                                                          acc[mt], 0, 0, 0);
        } else if constexpr (KIND == GemmKind::F16) {
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[u][mt]),
                                                           __builtin_bit_cast(f16x8, bf[u]),
                                                           acc[mt], 0, 0, 0);
        } else {
          const f32x4 x0 = __builtin_bit_cast(f32x4, af[u][mt]);
          const f32x4 x1 = __builtin_bit_cast(f32x4, af2[u][mt]);
          f16x8 hi, lo;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hi[e] = (_Float16)x0[e];
            hi[4 + e] = (_Float16)x1[e];
            lo[e] = (_Float16)(x0[e] - (float)hi[e]);
            lo[4 + e] = (_Float16)(x1[e] - (float)hi[4 + e]);
          }
          const f16x8 bb = __builtin_bit_cast(f16x8, bf[u]);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bb, acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, bb, acc[mt], 0, 0, 0);
        }
      }
    }
  }

#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[w][mt][lane] = acc[mt];
  __syncthreads();

  // Epilogue: thread t -> (row, col) with col fastest (64-byte row segments).
  for (int o = threadIdx.x; o < 16 * MT * 16; o += 512) {
    const int col = o & 15;
    const int row = o >> 4;
    const int mt = row >> 4;
    const int rl = row & 15;
    const int src_lane = (rl >> 2) * 16 + col;
    const int reg = rl & 3;
    const int m = m0 + row;
    const int n = ntile * 16 + col;
    if (m >= a.M || n >= a.N) continue;
    if constexpr (KIND == GemmKind::I8) {
      int32_t s = 0;
#pragma unroll
      for (int ww = 0; ww < kGemmWaves; ++ww) s += red[ww][mt][src_lane][reg];
      const size_t idx = (size_t)m * a.N + n;
      if (a.acc_out) a.acc_out[idx] = s;
      if (a.C) {
        const float scale = (a.sa ? a.sa[m] : 1.f) * (a.sw ? a.sw[n] : 1.f);
        float y = __fmul_rn((float)s, scale);
        if (a.bias) y = __fadd_rn(y, a.bias[n]);
        a.C[idx] = apply_act(y, a.act);
      }
    } else {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < kGemmWaves; ++ww) s += red[ww][mt][src_lane][reg];
      if (a.bias) s += a.bias[n];
      a.C[(size_t)m * a.N + n] = apply_act(s, a.act);
    }
  }
}

// Repack W [K][N] (row-major) into per-(16-col tile, k-step) 1 KiB blocks,
// lane l's 16 bytes = W[k0 + (l>>4)*EPL + j][n0 + (l&15)], j < EPL
// (EPL = elements per lane: 16 int8 or 8 fp16); zero-padded past K / N.
template <typename T, int EPL>
__global__ void pack_kernel(const T* __restrict__ W, T* __restrict__ P, int K, int N, int KS,
                            int ntiles) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one lane-chunk
  const size_t total = (size_t)ntiles * KS * 64;
  if (idx >= total) return;
  const int lane = idx & 63;
  const size_t blk = idx >> 6;
  const int ks = blk % KS;
  const int nt = blk / KS;
  const int n = nt * 16 + (lane & 15);
  const int kb = ks * (4 * EPL) + (lane >> 4) * EPL;
  T* dst = P + idx * EPL;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int k = kb + j;
    dst[j] = (k < K && n < N) ? W[(size_t)k * N + n] : T(0);
  }
}

namespace {

template <GemmKind KIND>
hipError_t launch_gemm(const GemmArgs& a, hipStream_t st) {
  const int ntiles = (a.N + 15) / 16;
  const dim3 block(512);
  if (a.M <= 16) {
    hipLaunchKernelGGL((gemm_kernel<KIND, 1>), dim3(ntiles, 1), block, 0, st, a);
  } else if (a.M <= 32) {
    hipLaunchKernelGGL((gemm_kernel<KIND, 2>), dim3(ntiles, 1), block, 0, st, a);
  } else {
    hipLaunchKernelGGL((gemm_kernel<KIND, 4>), dim3(ntiles, (a.M + 63) / 64), block, 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace
}  // namespace llm

using namespace llm;

extern "C" size_t gemm_packed_bytes(int dtype, int K, int N) {
  if (K <= 0 || N <= 0) return 0;
  const int kstep = dtype == LLM_I8 ? 64 : 32;
  const size_t KS = (size_t)(K + kstep - 1) / kstep;
  const size_t nt = (size_t)(N + 15) / 16;
  return nt * KS * 1024;
}

extern "C" int gemm_pack_weights(int dtype, const void* W_kn, void* W_packed, int K, int N,
                                 void* stream) {
  LLM_REQUIRE(W_kn && W_packed && K > 0 && N > 0, "gemm_pack_weights: bad arguments");
  LLM_REQUIRE(dtype == LLM_I8 || dtype == LLM_F16, "gemm_pack_weights: dtype must be I8 or F16");
  const int kstep = dtype == LLM_I8 ? 64 : 32;
  const int KS = (K + kstep - 1) / kstep;
  const int ntiles = (N + 15) / 16;
  const size_t total = (size_t)ntiles * KS * 64;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = as_stream(stream);
  if (dtype == LLM_I8)
    hipLaunchKernelGGL((pack_kernel<int8_t, 16>), grid, dim3(256), 0, st,
                       static_cast<const int8_t*>(W_kn), static_cast<int8_t*>(W_packed), K, N, KS,
                       ntiles);
  else
    hipLaunchKernelGGL((pack_kernel<uint16_t, 8>), grid, dim3(256), 0, st,
                       static_cast<const uint16_t*>(W_kn), static_cast<uint16_t*>(W_packed), K, N,
                       KS, ntiles);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}

extern "C" int i8_gemm(const int8_t* A, int lda, const void* W_packed, int32_t* acc_out, float* C,
                       int M, int N, int K, const float* sa, const float* sw, const float* bias,
                       int act, void* stream) {
  LLM_REQUIRE(M >= 0 && N > 0 && K > 0, "i8_gemm: bad M/N/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(A && W_packed, "i8_gemm: NULL operand");
  LLM_REQUIRE(K % 64 == 0, "i8_gemm: K must be a multiple of 64");
  LLM_REQUIRE(N % 16 == 0, "i8_gemm: N must be a multiple of 16");
  LLM_REQUIRE(lda >= K && lda % 16 == 0, "i8_gemm: lda must be >= K and a multiple of 16");
  LLM_REQUIRE(act >= 0 && act <= 2, "i8_gemm: bad activation");
  LLM_REQUIRE((size_t)M * lda < (1ull << 31), "i8_gemm: A too large");
  GemmArgs a{};
  a.A = reinterpret_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.sa = sa; a.sw = sw; a.bias = bias; a.act = act;
  a.C = C; a.acc_out = acc_out;
  hipError_t e = launch_gemm<GemmKind::I8>(a, as_stream(stream));
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("i8_gemm: ") + hipGetErrorString(e));
  return LLM_OK;
}

extern "C" int f16_gemm(const void* A, int lda, const void* W_packed, float* C, int M, int N,
                        int K, const float* bias, int act, void* stream) {
  LLM_REQUIRE(M >= 0 && N > 0 && K > 0, "f16_gemm: bad M/N/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(A && W_packed && C, "f16_gemm: NULL operand");
  LLM_REQUIRE(K % 32 == 0, "f16_gemm: K must be a multiple of 32");
  LLM_REQUIRE(N % 16 == 0, "f16_gemm: N must be a multiple of 16");
  LLM_REQUIRE(lda >= K && lda % 8 == 0, "f16_gemm: lda must be >= K and a multiple of 8");
  LLM_REQUIRE(act >= 0 && act <= 2, "f16_gemm: bad activation");
  LLM_REQUIRE((size_t)M * lda * 2 < (1ull << 31), "f16_gemm: A too large");
  GemmArgs a{};
  a.A = static_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 32;
  a.bias = bias; a.act = act; a.C = C;
  hipError_t e = launch_gemm<GemmKind::F16>(a, as_stream(stream));
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("f16_gemm: ") + hipGetErrorString(e));
  return LLM_OK;
}

extern "C" int lm_head(const float* x, const void* E, float* logits, int M, int V, int K,
                       void* stream) {
  LLM_REQUIRE(M >= 0 && V > 0 && K > 0, "lm_head: bad M/V/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(x && E && logits, "lm_head: NULL operand");
  LLM_REQUIRE(K % 32 == 0, "lm_head: K must be a multiple of 32");
  LLM_REQUIRE((size_t)V * K * 2 < (1ull << 32) && (size_t)M * K * 4 < (1ull << 31),
              "lm_head: operands too large for 32-bit offsets");
  GemmArgs a{};
  a.A = reinterpret_cast<const uint8_t*>(x);
  a.lda = K;
  a.B = static_cast<const uint8_t*>(E);
  a.M = M; a.N = V; a.K = K; a.KS = K / 32;
  a.C = logits;
  hipError_t e = launch_gemm<GemmKind::LMHEAD>(a, as_stream(stream));
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("lm_head: ") + hipGetErrorString(e));
  return LLM_OK;
}
