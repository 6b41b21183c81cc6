// Tied-embedding LM head + greedy argmax for decode (logits = x . E^T, the
// LM head the reference lacks: SURVEY Appendix A #20; argmax = sample_from_logits,
// decoder/cuda_decoder.cu:7-14).
//
// x is fp32 [M][K] (M <= 64 per row block), E fp16 [V][K] row-major (the
// embedding table itself, read once per step: V*K*2 bytes, HBM-bound).
// To keep ~fp32 accuracy x is split into fp16 hi + lo and each E fragment
// feeds two v_mfma_f32_16x16x32_f16.
//
// Layout of the work: one workgroup = 8 waves = 128 vocabulary rows of E
// (each wave one 16-row tile), all M rows of x.  x is the operand every
// workgroup shares: it is staged per 256-wide K chunk into LDS once per
// workgroup (converted to hi/lo A fragments on the way), so the per-CU
// traffic is E once plus x once per 128 vocabulary rows, instead of x once
// per 16-32 rows as in a plain tile GEMM (the previous form: 146 us at C3).
// E fragments for the next chunk are in flight while the current one is
// multiplied.
//
// The epilogue writes the logits and a per-(row, workgroup) (max, first
// index) pair; argmax_partials_kernel reduces those pairs per row (first
// maximum wins), so greedy decoding never re-reads the [M][V] logits.
#include "common.hpp"
#include "row_ops.hpp"

namespace llm {

constexpr int kLmWaves = 8;
constexpr int kLmCols = 16 * kLmWaves;  // vocabulary rows per workgroup
constexpr int kLmKChunk = 256;          // K per LDS stage (8 k-steps of 32)
constexpr int kLmKs = kLmKChunk / 32;

struct LmHeadArgs {
  const float* x;
  const _Float16* E;
  float* logits;      // [M][V] (may be NULL when only the argmax is wanted)
  float* part_val;    // [M][nwg] max per (row, workgroup), or NULL
  int32_t* part_idx;  // [M][nwg]
  int M, V, K, nwg;
};

// MT = 16-row tiles of x per workgroup (1, 2 or 4).
template <int MT>
__global__ __launch_bounds__(512) void lm_head_kernel(LmHeadArgs a) {
  // A fragments of the chunk: [mt][ks][hi/lo][64 lanes] x 16 B
  __shared__ __attribute__((aligned(16))) u32x4 xa[MT][kLmKs][2][64];
  __shared__ float pv[kLmWaves][16 * MT];
  __shared__ int pi[kLmWaves][16 * MT];
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int m0 = blockIdx.y * 16 * MT;
  const int n0 = blockIdx.x * kLmCols + w * 16;  // this wave's 16 vocabulary rows
  const int nrow = n0 + (lane & 15);
  const int kg = lane >> 4;
  const auto ers = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.E, (short)0, (uint32_t)min((size_t)a.V * a.K * 2, (size_t)0xFFFFFFF0u), 0x00020000);
  const uint32_t e_off = nrow < a.V ? (uint32_t)((size_t)nrow * a.K * 2) + kg * 16 : 0xFFFFFFF0u;

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = (a.K + kLmKChunk - 1) / kLmKChunk;  // K % 32 == 0; tail k-steps load 0
  u32x4 eb[2][kLmKs];
  auto issue = [&](u32x4 (&dst)[kLmKs], int c) {
#pragma unroll
    for (int ks = 0; ks < kLmKs; ++ks) {
      const int k = c * kLmKChunk + ks * 32;
      const uint32_t off = (e_off == 0xFFFFFFF0u || k >= a.K) ? 0xFFFFFFF0u : e_off + (uint32_t)k * 2;
      dst[ks] = __builtin_amdgcn_raw_buffer_load_b128(ers, off, 0, 2);  // E: read once, nt
    }
  };
  // Stage x[m0:m0+16MT][c*256 : +256] as hi/lo A fragments: fragment (mt, ks)
  // lane l holds row mt*16 + (l&15), k = ks*32 + 8*(l>>4) .. +8.
  auto stage_x = [&](int c) {
    constexpr int FR = MT * kLmKs * 64;  // (mt, ks, lane) fragments of 8 values
    for (int f = threadIdx.x; f < FR; f += 512) {
      const int l = f & 63, ks = (f >> 6) % kLmKs, mt = (f >> 6) / kLmKs;
      const int row = m0 + mt * 16 + (l & 15);
      const int k = c * kLmKChunk + ks * 32 + 8 * (l >> 4);
      f32x4 v0{0.f, 0.f, 0.f, 0.f}, v1{0.f, 0.f, 0.f, 0.f};
      if (row < a.M && k < a.K) {
        const f32x4* src = reinterpret_cast<const f32x4*>(a.x + (size_t)row * a.K + k);
        v0 = src[0];
        v1 = src[1];
      }
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (_Float16)v0[e];
        hi[4 + e] = (_Float16)v1[e];
        lo[e] = (_Float16)(v0[e] - (float)hi[e]);
        lo[4 + e] = (_Float16)(v1[e] - (float)hi[4 + e]);
      }
      xa[mt][ks][0][l] = __builtin_bit_cast(u32x4, hi);
      xa[mt][ks][1][l] = __builtin_bit_cast(u32x4, lo);
    }
  };

  issue(eb[0], 0);
  for (int c = 0; c < nchunks; ++c) {
    stage_x(c);
    __syncthreads();
    if (c + 1 < nchunks) issue(eb[(c + 1) & 1], c + 1);
    const u32x4(&cur)[kLmKs] = eb[c & 1];
#pragma unroll
    for (int ks = 0; ks < kLmKs; ++ks) {
      const f16x8 bb = __builtin_bit_cast(f16x8, cur[ks]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f16x8 hi = __builtin_bit_cast(f16x8, xa[mt][ks][0][lane]);
        const f16x8 lo = __builtin_bit_cast(f16x8, xa[mt][ks][1][lane]);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bb, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, bb, acc[mt], 0, 0, 0);
      }
    }
    __syncthreads();  // xa is rewritten by the next chunk
  }

  // acc[mt] lane l, reg r: x row m0 + mt*16 + 4*(l>>4) + r, vocab row n0 + (l&15)
  // (C/D layout: col = lane&15 -> here the vocabulary index, row = 4*(lane>>4)+reg).
  const int n = n0 + (lane & 15);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + 4 * (lane >> 4) + r;
      const float v = acc[mt][r];
      if (a.logits && m0 + row < a.M && n < a.V) a.logits[(size_t)(m0 + row) * a.V + n] = v;
      if (a.part_val) {
        // max over this wave's 16 vocabulary rows (lanes sharing lane>>4), first index on ties
        float bv = n < a.V ? v : -INFINITY;
        int bi = n < a.V ? n : 0x7fffffff;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          const float ov = __shfl_xor(bv, off, 64);
          const int oi = __shfl_xor(bi, off, 64);
          if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if ((lane & 15) == 0) { pv[w][row] = bv; pi[w][row] = bi; }
      }
    }
  }
  if (!a.part_val) return;
  __syncthreads();
  for (int row = threadIdx.x; row < 16 * MT; row += 512) {
    if (m0 + row >= a.M) continue;
    float bv = pv[0][row];
    int bi = pi[0][row];
    for (int ww = 1; ww < kLmWaves; ++ww)  // waves cover increasing vocabulary rows
      if (pv[ww][row] > bv) { bv = pv[ww][row]; bi = pi[ww][row]; }
    a.part_val[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bv;
    a.part_idx[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bi;
  }
}

// Per row: the first maximum over the workgroup partials (in vocabulary order).
__global__ __launch_bounds__(256) void argmax_partials_kernel(const float* __restrict__ pv,
                                                              const int32_t* __restrict__ pi,
                                                              int nwg, int32_t* __restrict__ out) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int r = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = threadIdx.x; j < nwg; j += 256) {
    const float v = pv[(size_t)r * nwg + j];
    const int i = pi[(size_t)r * nwg + j];
    if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = bv; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    bv = sv[0];
    bi = si[0];
    for (int k = 1; k < 4; ++k)
      if (sv[k] > bv || (sv[k] == bv && si[k] < bi)) { bv = sv[k]; bi = si[k]; }
    out[r] = bi == 0x7fffffff ? 0 : bi;
  }
}

int lm_head_workgroups(int V) { return (V + kLmCols - 1) / kLmCols; }

hipError_t launch_lm_head(const float* x, const void* E, float* logits, int M, int V, int K,
                          float* part_val, int32_t* part_idx, hipStream_t st) {
  LmHeadArgs a{x, static_cast<const _Float16*>(E), logits, part_val, part_idx, M, V, K,
               lm_head_workgroups(V)};
  const int mt = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const dim3 grid(a.nwg, (M + 16 * mt - 1) / (16 * mt)), block(512);
  if (mt == 1) hipLaunchKernelGGL(lm_head_kernel<1>, grid, block, 0, st, a);
  else if (mt == 2) hipLaunchKernelGGL(lm_head_kernel<2>, grid, block, 0, st, a);
  else hipLaunchKernelGGL(lm_head_kernel<4>, grid, block, 0, st, a);
  return hipGetLastError();
}

hipError_t launch_argmax_partials(const float* part_val, const int32_t* part_idx, int M, int nwg,
                                  int32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(argmax_partials_kernel, dim3(M), dim3(256), 0, st, part_val, part_idx, nwg,
                     out);
  return hipGetLastError();
}

}  // namespace llm

using namespace llm;

extern "C" int lm_head(const float* x, const void* E, float* logits, int M, int V, int K,
                       void* stream) {
  LLM_REQUIRE(M >= 0 && V > 0 && K > 0, "lm_head: bad M/V/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(x && E && logits, "lm_head: NULL operand");
  LLM_REQUIRE(K % 32 == 0, "lm_head: K must be a multiple of 32");
  LLM_REQUIRE((size_t)V * K * 2 < 0xFFFFFFF0ull, "lm_head: E too large for 32-bit offsets");
  LLM_HIP_RET(launch_lm_head(x, E, logits, M, V, K, nullptr, nullptr, as_stream(stream)));
  return LLM_OK;
}
