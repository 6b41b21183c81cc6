// Tied-embedding LM head + greedy argmax for decode (logits = x . E^T, the
// LM head the reference lacks: SURVEY Appendix A #20; argmax = sample_from_logits,
// decoder/cuda_decoder.cu:7-14).
//
// x is fp32 [M][K] (M <= 64 per row block).  E fp16 [V][K] is the embedding
// table; the LM head streams a copy repacked once at load time into MFMA
// B-fragment order (lm_head_pack_embedding: one contiguous 1 KiB block per
// (16 vocabulary rows, 32-wide k-step)), read once per step with fully
// coalesced loads: V*K*2 bytes, HBM-bound.
// To keep ~fp32 accuracy x is split into fp16 hi + lo and each E fragment
// feeds two v_mfma_f32_16x16x32_f16.
//
// Layout of the work: one workgroup = 16 waves = 256 vocabulary rows of E
// (each wave one 16-row tile), all M rows of x.  x is the operand every
// workgroup shares: it is staged per 256-wide K chunk into LDS once per
// workgroup (converted to hi/lo A fragments on the way), so the per-CU
// traffic is E once plus x once per 256 vocabulary rows, instead of x once
// per 16-32 rows as in a plain tile GEMM (the previous form: 146 us at C3).
// Registers (scripts/kernel_resources.sh, gfx950): lm_head_kernel<1|2|4>
// (M tiles of 16 rows) use 100 / 104 / 124 VGPRs with no scratch, inside the
// 128 that __launch_bounds__(1024) leaves.
// E fragments for the next chunk are in flight while the current one is
// multiplied.
//
// The epilogue writes the logits and a per-(row, workgroup) (max, first
// index) pair; argmax_partials_kernel reduces those pairs per row (first
// maximum wins), so greedy decoding never re-reads the [M][V] logits.
#include "common.hpp"
#include "row_ops.hpp"

#include <algorithm>
#include <cstdlib>

namespace llm {

// 16 waves = 256 vocabulary rows per workgroup: x is staged once per 256 rows
// instead of 128, halving its share of the per-CU traffic (rocprof, C3 shape,
// scripts/time_lm_head.py: 57.6 vs 73.3 us per launch, identical logits; M 16 /
// 32 / 64 at K 768-2048: 16.2 vs 16.7, 45.2 vs 47.0, 24.2 vs 32.4 us)
// Vocabulary tiles per workgroup (LmHeadArgs::tiles, <= 16: waves past it only
// help stage x): the fewest that still give every CU at most ONE workgroup, so
// no CU streams more than its share of E -- for V = 50257 (3142 tiles) 13 per
// workgroup = 242 workgroups on 256 CUs, where 16 left 59 CUs idle (197
// workgroups of 1 MiB of E each at C3).  At least 8, so small vocabularies do
// not stage x once per tile.
constexpr int kLmWaves = 16;            // vocabulary tiles per workgroup <= 16
constexpr int kLmKChunk = 256;          // K per LDS stage (8 k-steps of 32)
constexpr int kLmKs = kLmKChunk / 32;

struct LmHeadArgs {
  const float* x;
  const _Float16* E;  // packed: [V/16][K/32][64 lanes][8]
  float* logits;      // [M][V] (may be NULL when only the argmax is wanted)
  float* part_val;    // [M][nwg] max per (row, workgroup), or NULL
  int32_t* part_idx;  // [M][nwg]
  int M, V, K, nwg;
  int tiles;  // vocabulary tiles (computing waves) per workgroup, <= kLmWaves
  int mode;  // 0; tuning build (LLM_LM_MODE): bit0 skip MFMA, bit1 skip x staging, bit2 skip
             // E loads; bit3: E with the default cache policy (kept) instead of nt
};

// MT = 16-row tiles of x per workgroup (1, 2 or 4); WAVES waves, each NTW
// vocabulary tiles (16 rows of E) per k-step against one read of the x
// fragments from LDS.
template <int MT, int WAVES, int NTW>
__global__ __launch_bounds__(WAVES * 64) void lm_head_kernel(LmHeadArgs a) {
  constexpr int kLmThreads = WAVES * 64;
  // A fragments of the chunk: [mt][ks][hi/lo][64 lanes] x 16 B
  __shared__ __attribute__((aligned(16))) u32x4 xa[MT][kLmKs][2][64];
  __shared__ float pv[WAVES * NTW][16 * MT];
  __shared__ int pi[WAVES * NTW][16 * MT];
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int m0 = blockIdx.y * 16 * MT;
  const int KS = a.K / 32;
  const int ntiles = (a.V + 15) / 16;
  const auto ers = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.E, (short)0, (uint32_t)min((size_t)ntiles * KS * 1024, (size_t)0xFFFFFFF0u), 0x00020000);
  // wave w's tiles: w * NTW + j of the workgroup's `tiles` (a wave past them only stages x)
  uint32_t e_off[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int t = w * NTW + j;
    const int ntile = blockIdx.x * a.tiles + t;
    e_off[j] = t < a.tiles && ntile < ntiles ? (uint32_t)((size_t)ntile * KS * 1024) + lane * 16
                                             : 0xFFFFFFF0u;
  }
  const bool mine = w * NTW < a.tiles;

  f32x4 acc[NTW][MT];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[j][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = (a.K + kLmKChunk - 1) / kLmKChunk;  // K % 32 == 0; tail k-steps load 0
  auto issue = [&](u32x4 (&dst)[NTW][kLmKs], int c) {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int ks = 0; ks < kLmKs; ++ks) {
        const int k = c * kLmKChunk + ks * 32;
        const uint32_t off =
            (e_off[j] == 0xFFFFFFF0u || k >= a.K) ? 0xFFFFFFF0u : e_off[j] + (uint32_t)(k / 32) * 1024u;
        dst[j][ks] = (a.mode & 4) ? u32x4{0u, 0u, 0u, (uint32_t)ks}
                     : (a.mode & 8) ? __builtin_amdgcn_raw_buffer_load_b128(ers, off, 0, 0)  // E kept
                                    : __builtin_amdgcn_raw_buffer_load_b128(ers, off, 0, 2);  // E: nt
      }
  };
  // Stage x[m0:m0+16MT][c*256 : +256] as hi/lo A fragments: fragment (mt, ks)
  // lane l holds row mt*16 + (l&15), k = ks*32 + 8*(l>>4) .. +8.  Each thread
  // owns FPT fragments; chunk c+1's x is loaded into registers while chunk c
  // is multiplied.
  constexpr int NFRAG = MT * kLmKs * 64;
  constexpr int FPT = (NFRAG + kLmThreads - 1) / kLmThreads;  // fragments per thread
  f32x4 xr[FPT][2];
  auto load_x = [&](int c) {
#pragma unroll
    for (int i = 0; i < FPT; ++i) {
      const int f = threadIdx.x + i * kLmThreads;
      const int l = f & 63, ks = (f >> 6) % kLmKs, mt = (f >> 6) / kLmKs;
      const int row = f < NFRAG ? m0 + mt * 16 + (l & 15) : a.M;
      const int k = c * kLmKChunk + ks * 32 + 8 * (l >> 4);
      xr[i][0] = xr[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < a.M && k < a.K && !(a.mode & 2)) {
        const f32x4* src = reinterpret_cast<const f32x4*>(a.x + (size_t)row * a.K + k);
        xr[i][0] = src[0];
        xr[i][1] = src[1];
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int i = 0; i < FPT; ++i) {
      const int f = threadIdx.x + i * kLmThreads;
      if (f >= NFRAG) break;
      const int l = f & 63, ks = (f >> 6) % kLmKs, mt = (f >> 6) / kLmKs;
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (_Float16)xr[i][0][e];
        hi[4 + e] = (_Float16)xr[i][1][e];
        lo[e] = (_Float16)(xr[i][0][e] - (float)hi[e]);
        lo[4 + e] = (_Float16)(xr[i][1][e] - (float)hi[4 + e]);
      }
      xa[mt][ks][0][l] = __builtin_bit_cast(u32x4, hi);
      xa[mt][ks][1][l] = __builtin_bit_cast(u32x4, lo);
    }
  };

  // One chunk: stage x, then multiply while the next chunk's E and x loads are
  // in flight.  The two E buffers are distinct named arrays (static register
  // indexing: a dynamically indexed register array would live in scratch).
  auto chunk = [&](const u32x4 (&cur)[NTW][kLmKs], u32x4 (&nxt)[NTW][kLmKs], int c) {
    store_x();
    __syncthreads();
    if (c + 1 < nchunks) {
      issue(nxt, c + 1);
      load_x(c + 1);
    }
    if (!mine) {
      // stages x only
    } else if (a.mode & 1) {
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        acc[j][0][0] += __builtin_bit_cast(float, cur[j][0][0] ^ cur[j][kLmKs - 1][3]) * 0.f +
                        (float)xa[0][0][0][lane][0];
    } else {
#pragma unroll
      for (int ks = 0; ks < kLmKs; ++ks) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f16x8 hi = __builtin_bit_cast(f16x8, xa[mt][ks][0][lane]);
          const f16x8 lo = __builtin_bit_cast(f16x8, xa[mt][ks][1][lane]);
#pragma unroll
          for (int j = 0; j < NTW; ++j) {
            const f16x8 bb = __builtin_bit_cast(f16x8, cur[j][ks]);
            acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bb, acc[j][mt], 0, 0, 0);
            acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, bb, acc[j][mt], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // xa is rewritten by the next chunk
  };
  u32x4 eA[NTW][kLmKs], eB[NTW][kLmKs];
  issue(eA, 0);
  load_x(0);
  for (int c = 0; c < nchunks; c += 2) {
    chunk(eA, eB, c);
    if (c + 1 < nchunks) chunk(eB, eA, c + 1);
  }

  // acc[j][mt] lane l, reg r: x row m0 + mt*16 + 4*(l>>4) + r, vocab row
  // 16 tile_j + (l&15) (C/D layout: col = lane&15 -> here the vocabulary
  // index, row = 4*(lane>>4)+reg).
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
  const int t = w * NTW + j;
  const int n = t < a.tiles ? (blockIdx.x * a.tiles + t) * 16 + (lane & 15) : a.V;  // staging-only: none
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + 4 * (lane >> 4) + r;
      const float v = acc[j][mt][r];
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
        if ((lane & 15) == 0 && t < WAVES * NTW) { pv[t][row] = bv; pi[t][row] = bi; }
      }
    }
  }
  }
  if (!a.part_val) return;
  __syncthreads();
  for (int row = threadIdx.x; row < 16 * MT; row += kLmThreads) {
    if (m0 + row >= a.M) continue;
    float bv = pv[0][row];
    int bi = pi[0][row];
    for (int ww = 1; ww < a.tiles; ++ww)  // tiles in increasing vocabulary order
      if (pv[ww][row] > bv) { bv = pv[ww][row]; bi = pi[ww][row]; }
    a.part_val[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bv;
    a.part_idx[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bi;
  }
}

// <= 16 rows with K <= 2048: x is staged into LDS ONCE for the whole K (hi / lo
// fragments, KS x 2 KiB of dynamic LDS) behind one barrier; then every wave
// streams its vocabulary tile's E with two 8-k-step batches in flight and no
// further barrier (lm_head_kernel stages x per 256-wide chunk, two barriers
// each, so every chunk waits for the workgroup's slowest E load).  Same
// MFMA sequence per tile (hi then lo, k ascending): the same logits bit for
// bit as lm_head_kernel<1, 16, 1>.
__global__ __launch_bounds__(1024) void lm_head_x1_kernel(LmHeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) u32x4 xs[];  // [KS][hi/lo][64 lanes]
  __shared__ float pv[kLmWaves][16];
  __shared__ int pi[kLmWaves][16];
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int m0 = blockIdx.y * 16;
  const int KS = a.K / 32;
  const int ntiles = (a.V + 15) / 16;
  const auto ers = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.E, (short)0, (uint32_t)min((size_t)ntiles * KS * 1024, (size_t)0xFFFFFFF0u), 0x00020000);
  const int ntile = blockIdx.x * a.tiles + w;
  const bool mine = w < a.tiles;  // a wave past `tiles` only stages x
  const uint32_t e_off =
      mine && ntile < ntiles ? (uint32_t)((size_t)ntile * KS * 1024) + lane * 16 : 0xFFFFFFF0u;
  constexpr int U = 8;
  u32x4 eA[U], eB[U];
  auto issue = [&](u32x4 (&d)[U], int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      const uint32_t off = (e_off == 0xFFFFFFF0u || k >= KS) ? 0xFFFFFFF0u : e_off + (uint32_t)k * 1024u;
      d[u] = __builtin_amdgcn_raw_buffer_load_b128(ers, off, 0, 2);  // E: read once, nt
    }
  };
  if (mine) issue(eA, 0);  // the first E batch is in flight while x is staged
  // x fragment (ks, lane l): row m0 + (l & 15), k = 32 ks + 8 (l >> 4) .. +8
  for (int f = threadIdx.x; f < KS * 64; f += 1024) {
    const int l = f & 63, ks = f >> 6;
    const int row = m0 + (l & 15);
    const int k = ks * 32 + 8 * (l >> 4);
    f32x4 x0{0.f, 0.f, 0.f, 0.f}, x1{0.f, 0.f, 0.f, 0.f};
    if (row < a.M) {
      const f32x4* src = reinterpret_cast<const f32x4*>(a.x + (size_t)row * a.K + k);
      x0 = src[0];
      x1 = src[1];
    }
    f16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hi[e] = (_Float16)x0[e];
      hi[4 + e] = (_Float16)x1[e];
      lo[e] = (_Float16)(x0[e] - (float)hi[e]);
      lo[4 + e] = (_Float16)(x1[e] - (float)hi[4 + e]);
    }
    xs[(ks * 2) * 64 + l] = __builtin_bit_cast(u32x4, hi);
    xs[(ks * 2 + 1) * 64 + l] = __builtin_bit_cast(u32x4, lo);
  }
  __syncthreads();
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  auto mm = [&](const u32x4 (&d)[U], int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      if (k >= KS) break;
      const f16x8 bb = __builtin_bit_cast(f16x8, d[u]);
      const f16x8 hi = __builtin_bit_cast(f16x8, xs[(k * 2) * 64 + lane]);
      const f16x8 lo = __builtin_bit_cast(f16x8, xs[(k * 2 + 1) * 64 + lane]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bb, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, bb, acc, 0, 0, 0);
    }
  };
  if (mine) {
    for (int k0 = 0; k0 < KS; k0 += 2 * U) {
      if (k0 + U < KS) issue(eB, k0 + U);
      mm(eA, k0);
      if (k0 + U >= KS) break;
      if (k0 + 2 * U < KS) issue(eA, k0 + 2 * U);
      mm(eB, k0 + U);
    }
  }
  // acc lane l, reg r: x row m0 + 4 (l >> 4) + r, vocabulary row 16 ntile + (l & 15)
  const int n = mine ? ntile * 16 + (lane & 15) : a.V;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * (lane >> 4) + r;
    const float v = acc[r];
    if (a.logits && m0 + row < a.M && n < a.V) a.logits[(size_t)(m0 + row) * a.V + n] = v;
    if (a.part_val) {
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
  if (!a.part_val) return;
  __syncthreads();
  if (threadIdx.x < 16 && m0 + (int)threadIdx.x < a.M) {
    const int row = threadIdx.x;
    float bv = pv[0][row];
    int bi = pi[0][row];
    for (int ww = 1; ww < a.tiles; ++ww)  // tiles in increasing vocabulary order
      if (pv[ww][row] > bv) { bv = pv[ww][row]; bi = pi[ww][row]; }
    a.part_val[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bv;
    a.part_idx[(size_t)(m0 + row) * a.nwg + blockIdx.x] = bi;
  }
}

// Per row: the first maximum over the workgroup partials (in vocabulary order).
// pos / ctx (optional): the decode step's position advance of the row, fused
// here instead of a launch of its own.
__global__ __launch_bounds__(256) void argmax_partials_kernel(const float* __restrict__ pv,
                                                              const int32_t* __restrict__ pi,
                                                              int nwg, int32_t* __restrict__ out,
                                                              int32_t* __restrict__ pos,
                                                              int32_t* __restrict__ ctx) {
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
    if (pos) {
      pos[r] += 1;
      ctx[r] += 1;
    }
  }
}

namespace {
int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0) {
      (void)hipGetLastError();
      cus = 256;
    }
  }
  return cus;
}
}  // namespace

int lm_head_tiles(int V) {
#if LLM_TUNING
  // tuning build: A/B of the tiles per workgroup.  Read once per process: a
  // decoder sizes its argmax partials (lm_nwg) at create, so the value must
  // not change under it between create and a launch.
  static const int forced = env_int("LLM_LM_TILES", 0);
  if (forced >= 1 && forced <= kLmWaves) return forced;
#endif
  const int ntiles = (V + 15) / 16;
  const int cus = cu_count();
  return std::min(kLmWaves, std::max(8, (ntiles + cus - 1) / cus));
}

int lm_head_workgroups(int V) {
  const int t = lm_head_tiles(V);
  return ((V + 15) / 16 + t - 1) / t;
}

// E [V][K] row-major -> B-fragment order: block (vocab tile t, k-step s) is
// 1 KiB; lane l holds E[16 t + (l & 15)][32 s + 8 (l >> 4) + j], j < 8.
__global__ void lm_pack_kernel(const _Float16* __restrict__ E, _Float16* __restrict__ P, int V,
                               int K) {
  const size_t KS = K / 32;
  const size_t total = (size_t)((V + 15) / 16) * KS * 64;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int lane = idx & 63;
    const size_t blk = idx >> 6;
    const int s = blk % KS;
    const int t = blk / KS;
    const int v = t * 16 + (lane & 15);
    const int k = s * 32 + 8 * (lane >> 4);
    u32x4 val{0u, 0u, 0u, 0u};
    if (v < V) val = *reinterpret_cast<const u32x4*>(E + (size_t)v * K + k);
    reinterpret_cast<u32x4*>(P)[idx] = val;
  }
}

size_t lm_head_packed_bytes(int V, int K) { return (size_t)((V + 15) / 16) * (K / 32) * 1024; }

hipError_t launch_lm_pack(const void* E, void* P, int V, int K, hipStream_t st) {
  const size_t total = lm_head_packed_bytes(V, K) / 16;
  const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(lm_pack_kernel, dim3(blocks), dim3(256), 0, st,
                     static_cast<const _Float16*>(E), static_cast<_Float16*>(P), V, K);
  return hipGetLastError();
}

hipError_t launch_lm_head(const float* x, const void* E, float* logits, int M, int V, int K,
                          float* part_val, int32_t* part_idx, hipStream_t st) {
#if LLM_TUNING
  static const int mode = [] {
    const char* v = std::getenv("LLM_LM_MODE");
    return v ? std::atoi(v) : 0;
  }();
#else
  constexpr int mode = 0;
#endif
  LmHeadArgs a{x, static_cast<const _Float16*>(E), logits, part_val, part_idx, M, V, K,
               lm_head_workgroups(V), lm_head_tiles(V), mode};
  const int mt = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const dim3 grid(a.nwg, (M + 16 * mt - 1) / (16 * mt));
  // 16 waves x 1 vocabulary tile.  The tuning build's LLM_LM_FORM=1 (8 waves x
  // 2 tiles: the x fragments read from LDS once per 2 tiles) measured slower
  // at every row count (C3 / C4 / C2 shapes 58.7 / 46.1 / 16.3 vs 56.0 / 43.8 /
  // 15.9 us, profiles/r03/lm_head_forms.txt): the LDS reads do not bound it.
#if LLM_TUNING
  if (env_int("LLM_LM_FORM", 0)) {
    if (mt == 1) hipLaunchKernelGGL((lm_head_kernel<1, 8, 2>), grid, dim3(512), 0, st, a);
    else if (mt == 2) hipLaunchKernelGGL((lm_head_kernel<2, 8, 2>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((lm_head_kernel<4, 8, 2>), grid, dim3(512), 0, st, a);
    return hipGetLastError();
  }
#endif
  if (mt == 1 && a.K <= 2048 && mode == 0) {
    const size_t lds = (size_t)(a.K / 32) * 2 * 64 * sizeof(u32x4);
    hipLaunchKernelGGL(lm_head_x1_kernel, grid, dim3(1024), lds, st, a);
  } else if (mt == 1) hipLaunchKernelGGL((lm_head_kernel<1, 16, 1>), grid, dim3(1024), 0, st, a);
  else if (mt == 2) hipLaunchKernelGGL((lm_head_kernel<2, 16, 1>), grid, dim3(1024), 0, st, a);
  else hipLaunchKernelGGL((lm_head_kernel<4, 16, 1>), grid, dim3(1024), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_argmax_partials(const float* part_val, const int32_t* part_idx, int M, int nwg,
                                  int32_t* out, hipStream_t st, int32_t* pos, int32_t* ctx) {
  hipLaunchKernelGGL(argmax_partials_kernel, dim3(M), dim3(256), 0, st, part_val, part_idx, nwg,
                     out, pos, ctx);
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
  LLM_REQUIRE(lm_head_packed_bytes(V, K) < 0xFFFFFFF0ull, "lm_head: E too large for 32-bit offsets");
  // one-shot entry: pack E into a scratch copy (the decoder packs once at load)
  hipStream_t st = as_stream(stream);
  void* P = nullptr;
  LLM_HIP_RET(hipMallocAsync(&P, lm_head_packed_bytes(V, K), st));
  hipError_t e = launch_lm_pack(E, P, V, K, st);
  if (e == hipSuccess) e = launch_lm_head(x, P, logits, M, V, K, nullptr, nullptr, st);
  (void)hipFreeAsync(P, st);
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("lm_head: ") + hipGetErrorString(e));
  return LLM_OK;
}
