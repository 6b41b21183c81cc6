// Paged decode attention for gfx950 (CDNA4).
//
// Replaces paged_flash_attention_kernel_fused / _overlap
// (attention/paged_flash_attention_kernel_fused.cu:5-90,
//  attention/paged_flash_attention_kernel_fused_overlap.cu:6-91) with the
// intended maths of cpu_paged_attention_forward
// (attention_cpu/cpu_attention_kernel.cpp:37-129).
//
// Decomposition (HBM-bound KV scan, ~1 flop/byte):
//   * one WAVE per (row b, head h, split s).  Every (b, h) gets the same
//     number of splits NS (a launch constant, sized so B*H*NS waves fill the
//     chip's resident wave slots exactly once: no second, ragged round), and
//     the split length is derived ON DEVICE from the row's live context,
//     pps_b = ceil(ntiles_b / NS) <= 128 pages, so a hipGraph captured once
//     stays balanced as the context grows.  A split's page ids are two
//     coalesced dword loads (lane j holds pages j and 64 + j), broadcast with
//     v_readlane.
//   * a page (tile) of TS tokens x D fp16 is contiguous; a wave reads it with
//     TS*D*2/1024 buffer_load_dwordx4 instructions of 1 KiB each (lane l ->
//     bytes 16l..16l+15): LPT = D/8 lanes hold one token row, TPI = 64/LPT
//     tokens per instruction.  K and V go straight to VGPRs: each byte is used
//     by exactly one wave, so an LDS round trip would be pure overhead
//     (cdna_hip_programming.md, "GEMV / M <= 16" row and Appendix B
//     "Attention decode").  Two register stages: the next chunk's loads are
//     in flight while the current chunk is computed.
//   * invalid pages (table -1, >= num_pages, past the split) use a buffer
//     descriptor with num_records = 0: the loads return zeros and touch no
//     memory; their tokens are masked.
//   * q.k: 8 fp32 FMAs per lane per token row, then a DPP butterfly across the
//     LPT lanes of the row (quad_perm / row_half_mirror / row_mirror), so every
//     lane of the row holds the score.
//   * online softmax per ROW GROUP (lanes sharing lane/LPT): each group keeps
//     its own running max m, sum l and 8 output dims in registers, so the
//     inner loop has no cross-row communication; groups are merged once at the
//     end (flash-decoding within the wave), splits are merged by
//     pa_merge_kernel (or written directly when there is one split).
//   * scores are kept in log2 units (q pre-scaled by sm_scale*log2(e)) so
//     every exponential is one v_exp_f32.
#include "common.hpp"
#include "ln_wave.hpp"
#include "pa_decode.hpp"
#include "row_ops.hpp"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace llm {

struct PaSplitArgs {
  const uint8_t* k_pool;
  const uint8_t* v_pool;
  const int32_t* page_table;
  const float* q;
  int q_stride;     // elements between consecutive rows b of q
  float* out;       // DIRECT: final output [B][H][D]
  float* part_acc;  // [B*H*nsplit][D]
  float* part_ml;   // [B*H*nsplit][2]
  const int32_t* beam_ids;
  const int32_t* context_lens;
  int B, H, T;
  int num_pages, num_beams, max_tiles;
  size_t page_stride;  // bytes from page p to page p + 1 (K and V pages may interleave)
  int pps;     // > 0: fixed pages per split (<= 128); 0: ceil(ntiles_b / nsplit)
  int nsplit;  // splits per (b, h) (grid)
  int group;   // rows per wave group (beam width): the group's rows for one (head, split)
               // run as adjacent waves of one workgroup, so pages the rows share (a
               // forked prefix) are fetched from HBM once and re-served from L2
  float qscale;
  int balance16;  // BEAM, dynamic splits: cost of a beam-private tile in 1/16ths of a
                  // shared tile (>= 16) for cost-balanced split boundaries; 0: off
  // WGM (workgroup merge): one workgroup of nsplit (<= 8) waves per (b, h); the
  // splits meet in LDS and wave 0 writes the merged head straight into the
  // o_proj input, no merge launch.  out16: fp16 [B][H*D] (packed-A order when
  // pack), out (if set): fp32 [B][H*D]
  _Float16* out16;
  int pack;
  int wgm;
  int beam4;  // row_group 4: pa_beam4_kernel (one wave per (group, head, split))
  // WGM, fused o_proj (PaRowOutputs::o_acc): o_acc[b][o_n] += o_h . W_o[h rows]
  // (counted fixed point, common.hpp oacc_term); the last head's adder of a
  // column stores o_x[b][n] and clears the column
  long long* o_acc;
  float* o_x;
  const _Float16* wo_heads;  // [H][D/8][o_n][8]
  int o_n;
  int* o_flag;  // set to 1 when a head's term was clamped (common.hpp oacc_term)
};

constexpr int kWgmMaxSplits = 8;  // one merge batch (pa_merge_row_kernel's kMergeBatch)
constexpr int kOprojMaxD = 128;   // fused o_proj: two W_o column slices of D fp16 in VGPRs

constexpr int kMaxPps = 128;     // page ids held in two registers per lane
constexpr int kMaxSplits = 128;  // split weights held in two registers per merge lane

// Split length of a row with `ntiles` live tiles.
__device__ __forceinline__ int row_pps(int pps_fixed, int nsplit, int ntiles) {
  if (pps_fixed > 0) return pps_fixed;
  return min(max((ntiles + nsplit - 1) / nsplit, 1), kMaxPps);
}

// Pages per register stage: CHUNK_BYTES of K+V in flight per wave per stage.
template <int PAGE_BYTES, int CHUNK_BYTES>
constexpr int pages_per_stage() {
  return (CHUNK_BYTES / (2 * PAGE_BYTES)) > 0 ? CHUNK_BYTES / (2 * PAGE_BYTES) : 1;
}

// KV element types of the pools (AttentionCUDA::forward's T in {__half, bf16,
// int8_t, float}, attention/attention_cuda.cu:58-94).  int8 is the raw value
// (KVTileCache<int8_t> stores and the kernel reads it as a number, no scale).
template <int KVT>
constexpr int kv_elem_bytes() {
  return KVT == LLM_F32 ? 4 : KVT == LLM_I8 ? 1 : 2;
}

// Element e of a lane's 16-byte KV piece as fp32.
template <int KVT>
__device__ __forceinline__ float kv_at(const u32x4& r, int e) {
  if constexpr (KVT == LLM_F16) {
    return (float)__builtin_bit_cast(f16x8, r)[e];
  } else if constexpr (KVT == LLM_BF16) {
    const uint32_t w = r[e >> 1];
    return __uint_as_float((e & 1) ? (w & 0xFFFF0000u) : (w << 16));
  } else if constexpr (KVT == LLM_F32) {
    return __uint_as_float(r[e]);
  } else {
    return (float)(((int32_t)r[e >> 2] << (24 - 8 * (e & 3))) >> 24);
  }
}

// A page must fill at least one wave-wide load (64 lanes x 16 B) and at most
// one 16 KiB register stage.
constexpr bool kv_shape_ok(int D, int TS, int es) {
  return TS * D * es >= 1024 && TS * D * es <= 16384;
}

// KV pages are read exactly once per step: stream them with the non-temporal
// cache policy (buffer_load ... nt), which keeps them from evicting the page
// table / q / partials from L2 and measured 0.73 -> 0.81 of 8 TB/s at C3
// (scripts/tune_attention.py, variants 0 vs 1).
constexpr int kKvLoadAux = 2;

// STAGES = register stages in flight per wave (2: the next chunk loads while
// the current one is computed; 1: latency hidden by occupancy alone).
// MIN_WAVES > 0 asks the compiler for that many waves per SIMD.
// BEAM: beam-aware KV prefetch for row_group == 4 (one workgroup = the 4
// beams of one sequence for one (head, split)).  When the 4 rows are valid and
// hold equal contexts, the leading chunks whose pages all 4 rows share (a
// forked prefix) are fetched ONCE per workgroup: each wave loads a quarter of
// the chunk, the quarters meet in LDS (double-buffered, one barrier per chunk,
// the next chunk's quarter in flight during the current chunk's math) and
// every wave runs its own softmax/AV over the full chunk from LDS.  The rest
// of the split (beam-private pages) takes the per-wave direct path.
// WGM: the workgroup-merge form (PaSplitArgs::wgm): blockDim = 64 * nsplit,
// one workgroup per (b, h), wave w = split w.
// OPROJ (WGM only): the fused o_proj of the FP16 decoder (PaSplitArgs::o_acc).
template <int D, int TS, bool DIRECT, int CHUNK_BYTES = 16384, int AUX = kKvLoadAux,
          int STAGES = 2, int MIN_WAVES = 0, bool LOAD_ONLY = false, bool BEAM = false,
          int KVT = LLM_F16, bool FULLPATH = true, bool WGM = false, bool OPROJ = false>
__global__ __launch_bounds__(WGM ? 64 * kWgmMaxSplits : 256)
__attribute__((amdgpu_waves_per_eu(MIN_WAVES > 0 ? MIN_WAVES : 1)))
void pa_split_kernel(PaSplitArgs a) {
  constexpr int ES = kv_elem_bytes<KVT>();
  constexpr int EPL = 16 / ES;  // elements per lane per 16-byte load
  constexpr int LPT = D / EPL;
  constexpr int TPI = 64 / LPT;
  constexpr int NI = TS / TPI;
  constexpr int PAGE_BYTES = TS * D * ES;
  constexpr int U = pages_per_stage<PAGE_BYTES, CHUNK_BYTES>();
  constexpr int NR = U * NI;
  static_assert(LPT >= 1 && LPT <= 64 && TS % TPI == 0 && NI >= 1, "bad D/TS");

  static_assert(!(WGM && (DIRECT || BEAM)), "the workgroup merge is a split form");
  static_assert(!OPROJ || (WGM && KVT == LLM_F16), "the fused o_proj is a workgroup-merge form");
  const int lane = lane_id();
  const int wid = blockIdx.x * (WGM ? a.nsplit : 4) + wave_id_uniform();
  const int G = BEAM ? 4 : WGM ? 1 : a.group;
  const int gi = wid % G;  // row within the group (fastest: adjacent waves)
  const int rest = wid / G;
  const int s = rest % a.nsplit;
  const int gh = rest / a.nsplit;
  const int h = gh % a.H;
  const int b = (gh / a.H) * G + gi;
  // BEAM: the shared path runs only when all 4 rows exist, route to a valid
  // page-table row and hold the same context (a uniform decision: every wave
  // of the workgroup evaluates the same 4 rows, before any early return).
  bool share = false;
  int grow[4] = {0, 0, 0, 0};  // BEAM: the group's page-table rows
  if constexpr (BEAM) {
    share = true;
    const int g0 = b - gi;
    int T0 = -1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int bi = g0 + i;
      if (bi >= a.B) { share = false; break; }
      const int ri = a.beam_ids ? a.beam_ids[bi] : bi;
      int Ti = a.context_lens ? a.context_lens[bi] : a.T;
      Ti = min(max(Ti, 0), a.T);
      if (ri < 0 || ri >= a.num_beams || (i > 0 && Ti != T0)) { share = false; break; }
      T0 = Ti;
      grow[i] = ri;
    }
  }
  if (b >= a.B) return;
  const int bh = b * a.H + h;
  const size_t pidx = (size_t)bh * a.nsplit + s;  // partial-state slot
  const int r = a.beam_ids ? a.beam_ids[b] : b;
  int Tb = a.context_lens ? a.context_lens[b] : a.T;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + TS - 1) / TS, a.max_tiles);
  int tile0, count;
  {
    const int pps = row_pps(a.pps, a.nsplit, ntiles);
    tile0 = s * pps;
    count = min(pps, ntiles - tile0);
  }
  if constexpr (BEAM) {
    // Cost-balanced splits: a split's beam-private tiles are loaded by every
    // wave (4x the per-wave bytes of a shared tile, which the workgroup loads
    // once), so equal tile counts leave the splits holding the private tail
    // slowest.  The group's shared prefix (leading tiles whose page ids agree
    // in all 4 rows) is found cooperatively, 64 tiles per round, and the
    // boundaries put equal cost (shared 16, private balance16) in each split.
    // Every input is uniform over the workgroup, so all splits of a row (one
    // workgroup each) derive the same partition.
    if (share && a.balance16 >= 16 && a.pps == 0 && a.nsplit > 1 && ntiles > 0) {
      __shared__ int pfx_lds[4][64];
      const int32_t* prow = a.page_table + ((size_t)grow[gi] * a.H + h) * a.max_tiles;
      int nsh_t = 0;
      for (int blk = 0;; blk += 64) {
        const int t = blk + lane;
        int id = -1;
        if (t < ntiles) {
          id = prow[t];
          if (id >= a.num_pages) id = -1;
        }
        pfx_lds[gi][lane] = id;
        __syncthreads();
        const bool eq = t < ntiles && pfx_lds[0][lane] == pfx_lds[1][lane] &&
                        pfx_lds[0][lane] == pfx_lds[2][lane] && pfx_lds[0][lane] == pfx_lds[3][lane];
        const uint64_t mk = __ballot(eq);
        __syncthreads();
        const int run = mk == ~0ull ? 64 : __builtin_ctzll(~mk);
        nsh_t = blk + run;
        if (run < 64 || blk + 64 >= ntiles) break;
      }
      nsh_t = min(nsh_t, ntiles);
      if (nsh_t > 0 && nsh_t < ntiles) {
        const long long A = 16, P = a.balance16, ns = a.nsplit;
        const long long C = A * nsh_t + P * (ntiles - nsh_t);
        auto start = [&](int k) -> int {  // first tile of split k
          if (k <= 0) return 0;
          if (k >= ns) return ntiles;
          const long long x = (C * k + ns - 1) / ns;
          if (x <= A * nsh_t) return (int)((x + A - 1) / A);
          return (int)min<long long>(ntiles, nsh_t + (x - A * nsh_t + P - 1) / P);
        };
        // every tile costs >= A, so no split holds more than C/ns/A + 2 tiles
        if ((C + ns - 1) / ns / A + 2 <= kMaxPps) {
          tile0 = start(s);
          count = start(s + 1) - tile0;
        }
      }
    }
  }
  const int c = lane % LPT;
  const int g = lane / LPT;

  if (count <= 0) {
    if constexpr (BEAM && !DIRECT) {
      // the merge of a beam launch reads every split: an empty one holds
      // (m, l, acc) = (sentinel, 0, 0)
      if (lane < LPT) {
        float* o = a.part_acc + pidx * D + c * EPL;
#pragma unroll
        for (int e = 0; e < EPL; e += 4) *reinterpret_cast<f32x4*>(o + e) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (lane == 0) {
        a.part_ml[pidx * 2] = kNegSentinel;
        a.part_ml[pidx * 2 + 1] = 0.f;
      }
    }
    if constexpr (DIRECT) {
      if (lane < LPT) {
        float* o = a.out + (size_t)bh * D + c * EPL;
#pragma unroll
        for (int e = 0; e < EPL; e += 4) *reinterpret_cast<f32x4*>(o + e) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if constexpr (!WGM) return;
    count = 0;  // WGM: no partial (the merge reads splits < ns only), but meet the workgroup
  }

  // Page ids of this split: lane j holds pages j and 64 + j
  // (PageTable::lookup semantics: out of range or >= num_pages -> missing).
  int pid0 = -1, pid1 = -1;
  if (r >= 0 && r < a.num_beams) {
    const int32_t* row = a.page_table + ((size_t)r * a.H + h) * a.max_tiles + tile0;
    if (lane < count) pid0 = row[lane];
    if (64 + lane < count) pid1 = row[64 + lane];
    if (pid0 >= a.num_pages) pid0 = -1;
    if (pid1 >= a.num_pages) pid1 = -1;
  }
  auto page_of = [&](int j) -> int {  // j is wave-uniform
    return j < 64 ? __builtin_amdgcn_readlane(pid0, j) : __builtin_amdgcn_readlane(pid1, min(j - 64, 63));
  };

  // q chunk of this lane (dims c*EPL .. c*EPL+EPL-1), pre-scaled into log2 units.
  float qv[EPL];
  {
    const float* qp = a.q + (size_t)b * a.q_stride + (size_t)h * D + c * EPL;
#pragma unroll
    for (int e0 = 0; e0 < EPL; e0 += 4) {
      const f32x4 qq = *reinterpret_cast<const f32x4*>(qp + e0);
#pragma unroll
      for (int e = 0; e < 4; ++e) qv[e0 + e] = qq[e] * a.qscale;
    }
  }

  float m = kNegSentinel, l = 0.f;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;

  const uint32_t lane_off = (uint32_t)lane * 16u;

  auto issue = [&](u32x4 (&kk)[NR], u32x4 (&vv)[NR], int p0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = p0 + u;
      const int pg = page_of(min(j, kMaxPps - 1));
      const bool ok = (j < count) && (pg >= 0);
      const size_t off = (size_t)(ok ? pg : 0) * a.page_stride;
      const auto krs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.k_pool + off), (short)0,
                                                         ok ? PAGE_BYTES : 0, 0x00020000);
      const auto vrs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.v_pool + off), (short)0,
                                                         ok ? PAGE_BYTES : 0, 0x00020000);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        kk[u * NI + i] = __builtin_amdgcn_raw_buffer_load_b128(krs, lane_off + i * 1024, 0, AUX);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        vv[u * NI + i] = __builtin_amdgcn_raw_buffer_load_b128(vrs, lane_off + i * 1024, 0, AUX);
    }
  };

  auto compute = [&](const u32x4 (&kk)[NR], const u32x4 (&vv)[NR], int p0) {
    if constexpr (LOAD_ONLY) {  // tuning: the same stream with a trivial consumer
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < NR; ++i) x ^= kk[i][0] ^ kk[i][3] ^ vv[i][1] ^ vv[i][2];
      acc[0] += (float)(x & 1u);
      return;
    }
    // One page u of the chunk.  FULL (wave-uniform): the page is present and
    // every one of its tokens is inside the context, so no token needs the
    // validity selects (the common case: all but a row's last page).
    auto page_math = [&](auto full_tag, int u, bool ok, int tok_base) {
      constexpr bool FULL = decltype(full_tag)::value;
      float sc[NI];
      bool valid[NI];
      float mloc = kNegSentinel;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < EPL; ++e) d = fmaf(qv[e], kv_at<KVT>(kk[u * NI + i], e), d);
        d = group_sum<LPT>(d);
        valid[i] = FULL || (ok && (tok_base + i * TPI) < Tb);
        sc[i] = valid[i] ? d : kNegSentinel;
        mloc = fmaxf(mloc, sc[i]);
      }
      const float mnew = fmaxf(m, mloc);
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      l *= corr;
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] *= corr;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float p = valid[i] ? __builtin_amdgcn_exp2f(sc[i] - mnew) : 0.f;
        l += p;
        // Rows past the context (or of a missing page) may hold stale bits, even
        // NaN/Inf in a never-written page: select them away (0 * NaN = NaN).
        const u32x4 vraw = FULL || valid[i] ? vv[u * NI + i] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < EPL; ++e) acc[e] = fmaf(p, kv_at<KVT>(vraw, e), acc[e]);
      }
      m = mnew;
    };
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = p0 + u;
      const int pg = page_of(min(j, kMaxPps - 1));
      const bool ok = (j < count) && (pg >= 0);
      const int tok_base = (tile0 + j) * TS + g;
      if (FULLPATH && ok && (tile0 + j + 1) * TS <= Tb)
        page_math(std::true_type{}, u, ok, tok_base);
      else
        page_math(std::false_type{}, u, ok, tok_base);
    }
  };

  const int nchunks = (count + U - 1) / U;
  int ch0 = 0;  // first chunk of the per-wave direct path
  if constexpr (BEAM) {
    static_assert(NR % 2 == 0, "beam prefetch splits a chunk's 2*NR pieces in quarters");
    constexpr int QP = NR / 2;  // pieces per wave per chunk
    __shared__ int pid_lds[4][128];
    __shared__ __attribute__((aligned(16))) u32x4 kvbuf[2][2 * NR][64];
    if (share) {
      pid_lds[gi][lane] = pid0;
      pid_lds[gi][64 + lane] = pid1;
      __syncthreads();
      const bool e0 = pid_lds[0][lane] == pid_lds[1][lane] && pid_lds[0][lane] == pid_lds[2][lane] &&
                      pid_lds[0][lane] == pid_lds[3][lane];
      const int l1 = 64 + lane;
      const bool e1 = pid_lds[0][l1] == pid_lds[1][l1] && pid_lds[0][l1] == pid_lds[2][l1] &&
                      pid_lds[0][l1] == pid_lds[3][l1];
      const uint64_t mk0 = __ballot(e0), mk1 = __ballot(e1);
      int nsh = 0;  // leading chunks whose pages are all shared (uniform)
      for (; nsh < nchunks; ++nsh) {
        bool all = true;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = nsh * U + u;
          if (j < count) all = all && (((j < 64 ? mk0 >> j : mk1 >> (j - 64)) & 1ull) != 0);
        }
        if (!all) break;
      }
      nsh = __builtin_amdgcn_readfirstlane(nsh);
      // this wave's quarter of chunk cc: pieces q = gi*QP + t of [K pieces | V pieces]
      auto quarter = [&](u32x4 (&qr)[QP], int cc) {
#pragma unroll
        for (int t = 0; t < QP; ++t) {
          const int q = gi * QP + t;
          const int pi = q % NR;
          const int u = pi / NI, i = pi % NI;
          const int j = cc * U + u;
          const int pg = page_of(min(j, kMaxPps - 1));
          const bool ok = (j < count) && (pg >= 0);
          const size_t off = (size_t)(ok ? pg : 0) * a.page_stride;
          const uint8_t* pool = q < NR ? a.k_pool : a.v_pool;
          const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(pool + off), (short)0,
                                                            ok ? PAGE_BYTES : 0, 0x00020000);
          qr[t] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + i * 1024, 0, AUX);
        }
      };
      if (nsh > 0) {
        u32x4 qr[QP];
        quarter(qr, 0);
#pragma unroll
        for (int t = 0; t < QP; ++t) kvbuf[0][gi * QP + t][lane] = qr[t];
        if (nsh > 1) quarter(qr, 1);
        __syncthreads();
        for (int cc = 0; cc < nsh; ++cc) {
          const int cur = cc & 1;
          u32x4 kk[NR], vv[NR];
#pragma unroll
          for (int p = 0; p < NR; ++p) {
            kk[p] = kvbuf[cur][p][lane];
            vv[p] = kvbuf[cur][NR + p][lane];
          }
          compute(kk, vv, cc * U);
          if (cc + 1 < nsh) {
            // buf[cur ^ 1] was last read in iteration cc - 1, before its barrier
#pragma unroll
            for (int t = 0; t < QP; ++t) kvbuf[cur ^ 1][gi * QP + t][lane] = qr[t];
            if (cc + 2 < nsh) quarter(qr, cc + 2);
          }
          __syncthreads();
        }
      }
      ch0 = nsh;
    }
  }
  if constexpr (STAGES == 1) {
    u32x4 kA[NR], vA[NR];
    for (int ch = ch0; ch < nchunks; ++ch) {
      issue(kA, vA, ch * U);
      compute(kA, vA, ch * U);
    }
  } else if (ch0 < nchunks) {
    u32x4 kA[NR], vA[NR], kB[NR], vB[NR];
    issue(kA, vA, ch0 * U);
    for (int ch = ch0; ch < nchunks; ch += 2) {
      issue(kB, vB, (ch + 1) * U);  // past-the-end chunks load nothing (num_records 0)
      compute(kA, vA, ch * U);
      if (ch + 1 >= nchunks) break;
      issue(kA, vA, (ch + 2) * U);
      compute(kB, vB, (ch + 1) * U);
    }
  }

  // Merge the TPI row groups of the wave (lanes with equal c).
#pragma unroll
  for (int off = LPT; off < 64; off <<= 1) {
    const float mo = __shfl_xor(m, off, 64);
    const float lo = __shfl_xor(l, off, 64);
    const float mn = fmaxf(m, mo);
    const float ca = __builtin_amdgcn_exp2f(m - mn);
    const float cb = __builtin_amdgcn_exp2f(mo - mn);
    l = l * ca + lo * cb;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const float ao = __shfl_xor(acc[e], off, 64);
      acc[e] = acc[e] * ca + ao * cb;
    }
    m = mn;
  }

  if constexpr (WGM) {
    // The workgroup's waves are the splits of one (b, h): their states meet in
    // LDS and wave 0 merges them with pa_merge_row_kernel's arithmetic (same
    // weights, same sequential order over splits 0..7, zero weights past ns),
    // so the o_proj input is bit-identical to the split + merge launches'.
    __shared__ float wg_ml[kWgmMaxSplits][2];
    __shared__ __attribute__((aligned(16))) float wg_acc[kWgmMaxSplits][D];
    if (lane < LPT) {
#pragma unroll
      for (int e = 0; e < EPL; e += 4)
        *reinterpret_cast<f32x4*>(&wg_acc[s][c * EPL + e]) =
            f32x4{acc[e], acc[e + 1], acc[e + 2], acc[e + 3]};
    }
    if (lane == 0) {
      wg_ml[s][0] = m;
      wg_ml[s][1] = l;
    }
    // OPROJ: wave s takes o_proj columns s*64 + lane + j*64*nsplit, CF columns
    // per round (CF * D fp16 = 128 VGPRs; each load instruction 1 KiB
    // contiguous); the first round's W_o slices are in flight across the merge
    constexpr int KG = D / 8;
    constexpr int CF = KG >= 32 ? 1 : 32 / KG;
    const int o_n = OPROJ ? a.o_n : 0;
    const int ocol0 = s * 64 + lane;
    const int ostride = 64 * a.nsplit;
    f16x8 wcur[OPROJ ? CF : 1][OPROJ ? KG : 1];
    auto load_round = [&](int base) {
#pragma unroll
      for (int j = 0; j < CF; ++j) {
        const f16x8* src = reinterpret_cast<const f16x8*>(a.wo_heads) + (size_t)h * KG * o_n +
                           min(base + j * ostride, o_n - 1);
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) wcur[j][kg] = src[(size_t)kg * o_n];
      }
    };
    if constexpr (OPROJ) load_round(ocol0);
    __syncthreads();
    if (!OPROJ && s != 0) return;
    __shared__ __attribute__((aligned(16))) _Float16 wg_o[OPROJ ? D : 8];
    if (s == 0) {
      const int pps = row_pps(a.pps, a.nsplit, ntiles);
      const int ns = min(a.nsplit, (ntiles + pps - 1) / pps);
      const float m0 = lane < ns ? wg_ml[lane][0] : kNegSentinel;
      const float l0 = lane < ns ? wg_ml[lane][1] : 0.f;
      const float M = ln_wave_max(fmaxf(m0, kNegSentinel));
      float o[EPL];
#pragma unroll
      for (int e = 0; e < EPL; ++e) o[e] = 0.f;
      if (ns > 0 && M > 0.5f * kNegSentinel) {
        const float w0 = lane < ns ? __builtin_amdgcn_exp2f(m0 - M) : 0.f;
        float L = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < kWgmMaxSplits; ++s2)
          if (s2 < ns) {
            const float ls = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l0), s2));
            const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));
            L += ls * ws;
          }
        const float inv = 1.0f / (L + 1e-6f);
        float am[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) am[e] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < kWgmMaxSplits; ++s2) {
          const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));  // 0 past ns
          const float* src = &wg_acc[min(s2, max(ns - 1, 0))][c * EPL];
#pragma unroll
          for (int e = 0; e < EPL; ++e) am[e] += src[e] * ws;
        }
#pragma unroll
        for (int e = 0; e < EPL; ++e) o[e] = am[e] * inv;
      }
      if (lane < LPT) {
        const int hid = a.H * D;
        const int k0 = h * D + c * EPL;
        if (a.out) {
          float* op = a.out + (size_t)b * hid + k0;
#pragma unroll
          for (int e = 0; e < EPL; e += 4) *reinterpret_cast<f32x4*>(op + e) = f32x4{o[e], o[e + 1], o[e + 2], o[e + 3]};
        }
        if (a.out16) {
          static_assert(KVT != LLM_F16 || EPL == 8, "fp16 lanes hold 8 dims: one 16-byte store");
          if constexpr (EPL == 8) {
            f16x8 pk;
#pragma unroll
            for (int e = 0; e < 8; ++e) pk[e] = (_Float16)o[e];
            *reinterpret_cast<f16x8*>(a.out16 + (a.pack ? a_frag_off_f16(b, k0, hid >> 5)
                                                        : (size_t)b * hid + k0)) = pk;
          }
        }
        if constexpr (OPROJ) {
#pragma unroll
          for (int e = 0; e < EPL; ++e) wg_o[c * EPL + e] = (_Float16)o[e];
        }
      }
    }  // s == 0
    if constexpr (OPROJ) {
      // o_acc[b][n] += sum_k o16[k] W_o[h D + k][n] for this wave's columns:
      // fp16 products, fp32 sums (v_dot2_f32_f16), one returning int64 atomic
      // per column (64 consecutive columns = 512 B per atomic instruction); the
      // adder that completes a column (H - 1 arrivals before it) stores the
      // row value x[b][n] and clears the column for the next layer
      __syncthreads();
      long long* orow = a.o_acc + (size_t)b * o_n;
      const f16x2* op = reinterpret_cast<const f16x2*>(wg_o);
      const float olim = oacc_limit(a.H);
      bool clamped = false;
      for (int base = ocol0; base < o_n; base += CF * ostride) {
        if (base != ocol0) load_round(base);
        float pj[CF];
#pragma unroll
        for (int j = 0; j < CF; ++j) {
          float p = 0.f;
#pragma unroll
          for (int kg = 0; kg < KG; ++kg)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              p = __builtin_amdgcn_fdot2(f16x2{wcur[j][kg][2 * e], wcur[j][kg][2 * e + 1]},
                                         op[kg * 4 + e], p, false);
          pj[j] = p;
        }
        // every column's atomic in flight before any result is used
        long long tj[CF], oj[CF];
#pragma unroll
        for (int j = 0; j < CF; ++j) {
          const int n = base + j * ostride;
          bool cj;
          tj[j] = oacc_term(pj[j], olim, cj);
          clamped |= cj && n < o_n;
          oj[j] = n < o_n ? (long long)atomicAdd(reinterpret_cast<unsigned long long*>(orow + n),
                                                 (unsigned long long)tj[j])
                          : 0;
        }
#pragma unroll
        for (int j = 0; j < CF; ++j) {
          const int n = base + j * ostride;
          if (n < o_n && oacc_count(oj[j]) == a.H - 1) {
            a.o_x[(size_t)b * o_n + n] = oacc_value(oj[j] + tj[j]);
            __hip_atomic_store(orow + n, 0LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      if (clamped) *a.o_flag = 1;
    }
    return;
  }

  if (lane < LPT) {
    if constexpr (DIRECT) {
      const float inv = 1.0f / (l + 1e-6f);
      float* o = a.out + (size_t)bh * D + c * EPL;
#pragma unroll
      for (int e = 0; e < EPL; e += 4)
        *reinterpret_cast<f32x4*>(o + e) =
            f32x4{acc[e] * inv, acc[e + 1] * inv, acc[e + 2] * inv, acc[e + 3] * inv};
    } else {
      float* o = a.part_acc + pidx * D + c * EPL;
#pragma unroll
      for (int e = 0; e < EPL; e += 4)
        *reinterpret_cast<f32x4*>(o + e) = f32x4{acc[e], acc[e + 1], acc[e + 2], acc[e + 3]};
      if (lane == 0) {
        a.part_ml[pidx * 2] = m;
        a.part_ml[pidx * 2 + 1] = l;
      }
    }
  }
}

#if LLM_TUNING
// Beam-group attention, one WAVE per (group of 4 beams, head, split): the
// wave loads each KV page ONCE into registers and runs the math of every beam
// that reads it (row_group 4, fp16 pools, pages <= 8 KiB).  A split's work is
// a list of page items: a page all 4 beams share (the group's leading tiles
// whose page ids agree in all 4 rows -- a forked prefix) is one item for all 4
// beams; a beam-private page is one item for its beam.  The items of a
// (group, head) are cut into nsplit equal runs (equal HBM bytes per wave:
// every item is one page), so no LDS, no barrier and no per-beam re-load;
// each beam keeps its own online-softmax state and the wave writes one split
// partial per beam, merged by pa_merge_row_kernel (every split holds one).
// Groups whose rows differ in context, route outside the table or do not all
// exist take the same kernel beam by beam (items of one beam, its own context,
// its own equal split of its tiles).
// Maths per beam as pa_split_kernel (log2 units, row groups of the wave merged
// at the end), so results match the plain schedule up to the split boundaries.
// MINW: waves per SIMD asked of the register allocator; U: page items per
// register stage (two stages in flight).
template <int D, int TS, int MINW = 2, int U = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MINW))) void pa_beam4_kernel(PaSplitArgs a) {
  constexpr int G = 4;
  constexpr int EPL = 8;  // fp16 elements per 16-byte lane load
  constexpr int LPT = D / EPL;
  constexpr int TPI = 64 / LPT;
  constexpr int NI = TS / TPI;
  constexpr int PAGE_BYTES = TS * D * 2;
  static_assert(LPT >= 1 && LPT <= 64 && TS % TPI == 0 && NI >= 1 && PAGE_BYTES <= 8192,
                "pa_beam4_kernel: fp16 pages of 1..8 KiB");
  const int lane = lane_id();
  const int wid = blockIdx.x * 4 + wave_id_uniform();
  const int s = wid % a.nsplit;
  const int gh = wid / a.nsplit;
  const int h = gh % a.H;
  const int grp = gh / a.H;
  if (grp >= (a.B + G - 1) / G) return;
  const int b0 = grp * G;
  const int c = lane % LPT;
  const int g = lane / LPT;

  // the group's rows (wave-uniform): page-table row, context, existence
  int prow_off[G], Tg[G];
  bool live[G];
  bool share = true;
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int bi = b0 + i;
    live[i] = bi < a.B;
    int ri = -1, Ti = 0;
    if (live[i]) {
      ri = a.beam_ids ? a.beam_ids[bi] : bi;
      Ti = a.context_lens ? a.context_lens[bi] : a.T;
      Ti = min(max(Ti, 0), a.T);
    }
    const bool rok = ri >= 0 && ri < a.num_beams;
    prow_off[i] = rok ? (ri * a.H + h) * a.max_tiles : -1;
    Tg[i] = rok ? Ti : 0;  // a row outside the table reads nothing (all pages missing)
    if (!live[i] || !rok || Ti != Tg[0]) share = false;
  }

  // q of each beam (dims c*8 .. c*8+7), pre-scaled into log2 units
  float qv[G][EPL];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const float* qp = a.q + (size_t)min(b0 + i, a.B - 1) * a.q_stride + (size_t)h * D + c * EPL;
    const f32x4 q0 = *reinterpret_cast<const f32x4*>(qp);
    const f32x4 q1 = *reinterpret_cast<const f32x4*>(qp + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qv[i][e] = q0[e] * a.qscale;
      qv[i][4 + e] = q1[e] * a.qscale;
    }
  }
  float m[G], l[G], acc[G][EPL];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    m[i] = kNegSentinel;
    l[i] = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[i][e] = 0.f;
  }
  const uint32_t lane_off = (uint32_t)lane * 16u;

  // One segment = a list of <= 128 page items, lane j holding item j and 64 + j
  // (page id, and tile << 4 | beam mask); shared groups have one segment,
  // the others one per beam.
  const int nseg = share ? 1 : G;
  for (int seg = 0; seg < nseg; ++seg) {
    int i0 = 0, cnt = 0, nsh = 0, ntiles = 0;
    if (share) {
      ntiles = min((Tg[0] + TS - 1) / TS, a.max_tiles);
      for (int blk = 0; blk < ntiles; blk += 64) {  // the shared prefix, 64 tiles per round
        const int t = blk + lane;
        bool eq = t < ntiles;
        if (eq) {
          const int32_t p0 = a.page_table[prow_off[0] + t];
#pragma unroll
          for (int i = 1; i < G; ++i) eq = eq && a.page_table[prow_off[i] + t] == p0;
        }
        const uint64_t mk = __ballot(eq);
        const int run = mk == ~0ull ? 64 : __builtin_ctzll(~mk);
        nsh = blk + run;
        if (run < 64) break;
      }
      nsh = min(nsh, ntiles);
      const int items = nsh + G * (ntiles - nsh);
      i0 = (int)(((long long)items * s) / a.nsplit);
      cnt = (int)(((long long)items * (s + 1)) / a.nsplit) - i0;
    } else {
      if (prow_off[seg] < 0) continue;  // no such row / outside the table: a neutral partial
      ntiles = min((Tg[seg] + TS - 1) / TS, a.max_tiles);
      const int pps = row_pps(0, a.nsplit, ntiles);
      i0 = s * pps;
      cnt = min(pps, ntiles - i0);
    }
    cnt = min(cnt, kMaxPps);  // the host sizes nsplit so a split holds <= 128 items
    if (cnt <= 0) continue;
    const int npriv = ntiles - nsh;
    int pid[2], inf[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int j = lane + 64 * r;
      pid[r] = -1;
      inf[r] = 0;
      if (j < cnt) {
        const int k = i0 + j;
        int tile, beam, mask;
        if (!share) {
          tile = k; beam = seg; mask = 1 << seg;
        } else if (k < nsh) {
          tile = k; beam = 0; mask = 0xF;
        } else {  // beam-major: a beam's private tiles are consecutive items
          const int p = k - nsh;
          beam = p / npriv; tile = nsh + p % npriv; mask = 1 << beam;
        }
        int id = a.page_table[prow_off[beam] + tile];
        pid[r] = id >= a.num_pages ? -1 : id;
        inf[r] = (tile << 4) | mask;
      }
    }
    auto item_pid = [&](int j) {
      return j < 64 ? __builtin_amdgcn_readlane(pid[0], j) : __builtin_amdgcn_readlane(pid[1], j - 64);
    };
    auto item_inf = [&](int j) {
      return j < 64 ? __builtin_amdgcn_readlane(inf[0], j) : __builtin_amdgcn_readlane(inf[1], j - 64);
    };
    auto issue = [&](u32x4 (&kk)[NI], u32x4 (&vv)[NI], int j) {
      const int pg = j < cnt ? item_pid(min(j, kMaxPps - 1)) : -1;
      const bool ok = pg >= 0;
      const size_t off = (size_t)(ok ? pg : 0) * a.page_stride;
      const auto krs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.k_pool + off), (short)0,
                                                         ok ? PAGE_BYTES : 0, 0x00020000);
      const auto vrs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.v_pool + off), (short)0,
                                                         ok ? PAGE_BYTES : 0, 0x00020000);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        kk[i] = __builtin_amdgcn_raw_buffer_load_b128(krs, lane_off + i * 1024, 0, kKvLoadAux);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        vv[i] = __builtin_amdgcn_raw_buffer_load_b128(vrs, lane_off + i * 1024, 0, kKvLoadAux);
    };
    // one page item for beam bi: scores, online softmax, p.v (pa_split_kernel maths)
    auto beam_math = [&](auto full_tag, auto beam_tag, const u32x4 (&kk)[NI],
                         const u32x4 (&vv)[NI], bool ok, int tok_base, int Tb) {
      constexpr bool FULL = decltype(full_tag)::value;
      constexpr int bi = decltype(beam_tag)::value;
      float sc[NI];
      bool valid[NI];
      float mloc = kNegSentinel;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < EPL; ++e) d = fmaf(qv[bi][e], kv_at<LLM_F16>(kk[i], e), d);
        d = group_sum<LPT>(d);
        valid[i] = FULL || (ok && (tok_base + i * TPI) < Tb);
        sc[i] = valid[i] ? d : kNegSentinel;
        mloc = fmaxf(mloc, sc[i]);
      }
      const float mnew = fmaxf(m[bi], mloc);
      const float corr = __builtin_amdgcn_exp2f(m[bi] - mnew);
      l[bi] *= corr;
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[bi][e] *= corr;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float p = valid[i] ? __builtin_amdgcn_exp2f(sc[i] - mnew) : 0.f;
        l[bi] += p;
        const u32x4 vraw = FULL || valid[i] ? vv[i] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < EPL; ++e) acc[bi][e] = fmaf(p, kv_at<LLM_F16>(vraw, e), acc[bi][e]);
      }
      m[bi] = mnew;
    };
    auto compute = [&](const u32x4 (&kk)[NI], const u32x4 (&vv)[NI], int j) {
      const int pg = item_pid(min(j, kMaxPps - 1));
      const int info = item_inf(min(j, kMaxPps - 1));
      const int tile = info >> 4, mask = info & 0xF;
      const bool ok = pg >= 0;
      const int Tb = share ? Tg[0] : Tg[seg];
      const bool full = ok && (tile + 1) * TS <= Tb;
      const int tok_base = tile * TS + g;
      auto each = [&](auto beam_tag) {
        constexpr int bi = decltype(beam_tag)::value;
        if (mask & (1 << bi)) {
          if (full)
            beam_math(std::true_type{}, beam_tag, kk, vv, ok, tok_base, Tb);
          else
            beam_math(std::false_type{}, beam_tag, kk, vv, ok, tok_base, Tb);
        }
      };
      each(std::integral_constant<int, 0>{});
      each(std::integral_constant<int, 1>{});
      each(std::integral_constant<int, 2>{});
      each(std::integral_constant<int, 3>{});
    };
    u32x4 kA[U][NI], vA[U][NI], kB[U][NI], vB[U][NI];
    auto issue_st = [&](u32x4 (&kk)[U][NI], u32x4 (&vv)[U][NI], int j0) {
#pragma unroll
      for (int u = 0; u < U; ++u) issue(kk[u], vv[u], j0 + u);  // past the end: no bytes
    };
    auto compute_st = [&](const u32x4 (&kk)[U][NI], const u32x4 (&vv)[U][NI], int j0) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j0 + u < cnt) compute(kk[u], vv[u], j0 + u);
    };
    issue_st(kA, vA, 0);
    for (int j = 0; j < cnt; j += 2 * U) {
      issue_st(kB, vB, j + U);
      compute_st(kA, vA, j);
      if (j + U >= cnt) break;
      issue_st(kA, vA, j + 2 * U);
      compute_st(kB, vB, j + U);
    }
  }

  // Per beam: merge the TPI row groups of the wave, write the split partial.
#pragma unroll
  for (int i = 0; i < G; ++i) {
#pragma unroll
    for (int off = LPT; off < 64; off <<= 1) {
      const float mo = __shfl_xor(m[i], off, 64);
      const float lo = __shfl_xor(l[i], off, 64);
      const float mn = fmaxf(m[i], mo);
      const float ca = __builtin_amdgcn_exp2f(m[i] - mn);
      const float cb = __builtin_amdgcn_exp2f(mo - mn);
      l[i] = l[i] * ca + lo * cb;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const float ao = __shfl_xor(acc[i][e], off, 64);
        acc[i][e] = acc[i][e] * ca + ao * cb;
      }
      m[i] = mn;
    }
    if (!live[i]) continue;
    const size_t pidx = ((size_t)(b0 + i) * a.H + h) * a.nsplit + s;
    if (lane < LPT) {
      float* o = a.part_acc + pidx * D + c * EPL;
      *reinterpret_cast<f32x4*>(o) = f32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{acc[i][4], acc[i][5], acc[i][6], acc[i][7]};
    }
    if (lane == 0) {
      a.part_ml[pidx * 2] = m[i];
      a.part_ml[pidx * 2 + 1] = l[i];
    }
  }
}
#endif  // LLM_TUNING

#if LLM_TUNING
// Tuning build only (LLM_BEAM_MFMA=1): measured slower than the VALU BEAM form
// it was written to replace (69.8 vs 60.8 us per C4 launch;
// loads alone 60.2 us, processing alone 48.3 us, both bound by what 2 waves
// per SIMD keep in flight).  Parity-green (fp32-grade against float64).
//
// MFMA beam-group kernel (row_group 4, fp16 KV, D 128, page 16): the 4 beams
// of a sequence for one (head, split) in one workgroup, as pa_split_kernel's
// BEAM form, but the q.k and p.v products run on the matrix cores, so a page
// costs the same few instructions whether it serves 1 beam or 4 (the VALU form
// spends 4 waves x ~90 instructions on every shared page: VALU/issue-bound,
// VERDICT r1).  Per page (16 tokens):
//   S^T[token][c] = K[token][:] . Qc[:]   4 x v_mfma_f32_16x16x32_f16; columns
//       c = b (beam b, q rounded to fp16) and c = 4 + b (the fp16 residual of
//       beam b's q, scaled by 2^13), summed with one lane shift: fp32-grade scores from
//       fp16 operands (K is fp16; products are exact in fp32)
//   online softmax per beam column in fp32 (the C layout puts a beam's 16
//       scores in 4 lanes x 4 registers)
//   O^T[d][c] += V^T[d][token] . P^T[token][c]   8 x v_mfma_f32_16x16x16_f16;
//       P^T is the score tile itself (same lanes: no movement), column b holding
//       fp16(p), column 4 + b the fp16 residual of p (summed once at the end);
//       V^T comes from a per-wave LDS image of the page read with
//       ds_read_b64_tr_b16 (the hardware transpose read), XOR-swizzled rows
// The 4 waves take the split's work items round-robin: a page all 4 beams
// share (leading shared run, as the BEAM form) is one item for all 4 beam
// columns; a beam-private page is one item masked to its beam.  Each item is
// loaded once, 1 KiB contiguous per instruction, into registers (two items in
// flight per wave), then into the wave's swizzled LDS images of K (read back
// as MFMA rows) and V (read back transposed).  The 4 waves' (m, l, acc) per beam
// are combined through LDS in a fixed order and written as the split's
// partial, which pa_merge_row_kernel consumes exactly as the VALU form's.
// Rows of a workgroup whose contexts differ (or that do not exist) fall back
// to one wave per beam with its own pages (items masked to that beam).
__device__ __forceinline__ uint32_t beam_lds_off(int row, int ch) {
  // 256-byte token rows, 16-byte chunk ch: XOR swizzle so the transposed reads
  // (4 rows x 32 bytes per 16-lane group) spread over the banks
  return (uint32_t)(256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))));
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Maximum over each 16-lane row (DPP, every lane of the row gets it).
__device__ __forceinline__ float row_max16(float x) {
  x = fmaxf(x, mov_dpp<0xB1>(x));   // quad_perm [1,0,3,2]
  x = fmaxf(x, mov_dpp<0x4E>(x));   // quad_perm [2,3,0,1]
  x = fmaxf(x, mov_dpp<0x141>(x));  // row_half_mirror
  return fmaxf(x, mov_dpp<0x140>(x));  // row_mirror
}
// The residual columns carry (x - fp16(x)) * 2^13: unscaled they would sit
// below fp16's normal range (~1e-5 for q, p * 2^-12 for the weights) and
// lose bits as subnormals.  Exact power-of-two scaling; |x| < 8192 keeps the
// scaled residual finite.  Measured against float64
// (scripts/debug_beam_mfma.py): 1.4e-7 .. 6.5e-7, as the VALU kernel.
// Values below fp16's smallest normal go to the residual column whole.
constexpr float kLoScale = 8192.f, kLoUnscale = 1.f / 8192.f;
constexpr float kF16MinNormal = 6.103515625e-05f;

// DBG (tuning build only): 1 = loads with a trivial consumer, 2 = processing
// with no loads (zero pages)
template <int DBG = 0>
__global__ __launch_bounds__(256) void pa_beam_mfma_kernel(PaSplitArgs a) {
  constexpr int D = 128, TS = 16;
  constexpr int PAGE_BYTES = TS * D * 2;  // 4 KiB
  __shared__ __attribute__((aligned(16))) uint8_t vimg[4][PAGE_BYTES];  // per wave
  __shared__ __attribute__((aligned(16))) uint8_t kimg[4][PAGE_BYTES];
  __shared__ __attribute__((aligned(16))) _Float16 pimg[4][16 * 16];
  __shared__ int pid_lds[4][kMaxPps];
  __shared__ int pfx_lds[4][64];

  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int s = blockIdx.x % a.nsplit;
  const int gh = blockIdx.x / a.nsplit;
  const int h = gh % a.H;
  const int g0 = (gh / a.H) * 4;
  const int b = g0 + w;  // this wave's beam row
  const bool brow = b < a.B;

  // share: all 4 rows exist, route to valid page-table rows and hold equal
  // contexts (uniform over the workgroup)
  bool share = true;
  int T0 = -1;
  for (int i = 0; i < 4; ++i) {
    const int bi = g0 + i;
    if (bi >= a.B) { share = false; break; }
    const int ri = a.beam_ids ? a.beam_ids[bi] : bi;
    int Ti = a.context_lens ? a.context_lens[bi] : a.T;
    Ti = min(max(Ti, 0), a.T);
    if (ri < 0 || ri >= a.num_beams || (i > 0 && Ti != T0)) { share = false; break; }
    T0 = Ti;
  }
  const int r = brow ? (a.beam_ids ? a.beam_ids[b] : b) : -1;
  int Tb = brow ? (a.context_lens ? a.context_lens[b] : a.T) : 0;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + TS - 1) / TS, a.max_tiles);
  int tile0, count;
  {
    const int pps = row_pps(a.pps, a.nsplit, ntiles);
    tile0 = s * pps;
    count = min(pps, ntiles - tile0);
  }
  const int32_t* prow =
      (r >= 0 && r < a.num_beams) ? a.page_table + ((size_t)r * a.H + h) * a.max_tiles : nullptr;
  if (share && a.balance16 >= 16 && a.pps == 0 && a.nsplit > 1 && ntiles > 0) {
    // cost-balanced split boundaries over the group's shared prefix (every
    // input uniform: all splits of the group derive the same partition)
    int nsh_t = 0;
    for (int blk = 0;; blk += 64) {
      const int t = blk + lane;
      int id = -1;
      if (t < ntiles) {
        id = prow[t];
        if (id >= a.num_pages) id = -1;
      }
      pfx_lds[w][lane] = id;
      __syncthreads();
      const bool eq = t < ntiles && pfx_lds[0][lane] == pfx_lds[1][lane] &&
                      pfx_lds[0][lane] == pfx_lds[2][lane] && pfx_lds[0][lane] == pfx_lds[3][lane];
      const uint64_t mk = __ballot(eq);
      __syncthreads();
      const int run = mk == ~0ull ? 64 : __builtin_ctzll(~mk);
      nsh_t = blk + run;
      if (run < 64 || blk + 64 >= ntiles) break;
    }
    nsh_t = min(nsh_t, ntiles);
    if (nsh_t > 0 && nsh_t < ntiles) {
      const long long A = 16, P = a.balance16, ns = a.nsplit;
      const long long C = A * nsh_t + P * (ntiles - nsh_t);
      auto start = [&](int k) -> int {
        if (k <= 0) return 0;
        if (k >= ns) return ntiles;
        const long long x = (C * k + ns - 1) / ns;
        if (x <= A * nsh_t) return (int)((x + A - 1) / A);
        return (int)min<long long>(ntiles, nsh_t + (x - A * nsh_t + P - 1) / P);
      };
      if ((C + ns - 1) / ns / A + 2 <= kMaxPps) {
        tile0 = start(s);
        count = start(s + 1) - tile0;
      }
    }
  }
  count = max(count, 0);

  // this split's page ids of every beam row of the group (-1: missing)
  for (int j = lane; j < kMaxPps; j += 64) {
    int id = -1;
    if (prow && j < count) {
      id = prow[tile0 + j];
      if (id >= a.num_pages) id = -1;
    }
    pid_lds[w][j] = id;
  }
  __syncthreads();

  // work items of this wave
  int nsh = 0, nitems, it0, istep;
  if (share) {
    while (nsh < count && pid_lds[0][nsh] == pid_lds[1][nsh] && pid_lds[0][nsh] == pid_lds[2][nsh] &&
           pid_lds[0][nsh] == pid_lds[3][nsh])
      ++nsh;
    nitems = nsh + 4 * (count - nsh);
    it0 = w;
    istep = 4;
  } else {
    nitems = count;
    it0 = 0;
    istep = 1;
  }
  nsh = __builtin_amdgcn_readfirstlane(nsh);
  // item -> (tile j, page, beam mask)
  auto item = [&](int i, int& j, int& pg, int& mask) {
    if (i >= nitems) { j = 0; pg = -1; mask = 0; return; }
    if (!share) { j = i; pg = pid_lds[w][j]; mask = 1 << w; return; }
    if (i < nsh) { j = i; pg = pid_lds[0][j]; mask = 0xF; return; }
    const int i2 = i - nsh;
    const int bb = i2 & 3;
    j = nsh + (i2 >> 2);
    pg = pid_lds[bb][j];
    mask = 1 << bb;
  };

  // q operands (A of the score MFMAs, rows = beams): lane row c = lane & 15,
  // c < 4: beam g0 + c, other rows 0; qh = fp16(q), ql = its fp16 residual
  // (scaled); k-step kk holds dims 32 kk + 8 (lane >> 4) .. + 7 (the K
  // operand's k order)
  const int col = lane & 15;
  const int lgrp = lane >> 4;
  f16x8 qh[4], ql[4];
  {
    const int qb = g0 + col;
    const bool qok = col < 4 && qb < a.B;
    const float* qp = a.q + (size_t)(qok ? qb : 0) * a.q_stride + (size_t)h * D;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = qok ? qp[32 * kk + 8 * lgrp + e] * a.qscale : 0.f;
        const _Float16 hi = fabsf(v) >= kF16MinNormal ? (_Float16)v : (_Float16)0.f;
        qh[kk][e] = hi;
        ql[kk][e] = (_Float16)((v - (float)hi) * kLoScale);
      }
    }
  }

  // online-softmax state of beam r in register r (lanes 0..15, identical)
  float m4[4], l4[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m4[r] = kNegSentinel;
    l4[r] = 0.f;
  }
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // P^T image of the wave: rows = beam columns (0..3 fp16(p), 4..7 residual,
  // 8..15 zero) x 16 tokens
  _Float16* pw = pimg[w];
  for (int i2 = 128 + lane; i2 < 256; i2 += 64) pw[i2] = (_Float16)0.f;
  uint8_t* vw = vimg[w];
  uint8_t* kw = kimg[w];

  struct Stage {
    u32x4 k[4], v[4];
  };
  auto issue = [&](Stage& st, int i) {
    int j, pg, mask;
    item(i, j, pg, mask);
    const bool ok = pg >= 0 && DBG != 2;
    const size_t off = (size_t)(ok ? pg : 0) * a.page_stride;
    const auto krs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.k_pool + off), (short)0,
                                                       ok ? PAGE_BYTES : 0, 0x00020000);
    const auto vrs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.v_pool + off), (short)0,
                                                       ok ? PAGE_BYTES : 0, 0x00020000);
    // K and V: linear 1 KiB per instruction (token 4 c + lgrp, chunk col)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      st.k[c] = __builtin_amdgcn_raw_buffer_load_b128(krs, (uint32_t)(c * 1024 + lane * 16), 0,
                                                       kKvLoadAux);
      st.v[c] = __builtin_amdgcn_raw_buffer_load_b128(vrs, (uint32_t)(c * 1024 + lane * 16), 0,
                                                       kKvLoadAux);
    }
  };
  auto process = [&](const Stage& st, int i) {
    if constexpr (DBG == 1) {
      uint32_t x = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) x ^= st.k[c][0] ^ st.v[c][3];
      acc[0][0] += (float)(x & 1u);
      return;
    }
    int j, pg, mask;
    item(i, j, pg, mask);
    const bool ok = pg >= 0;
    const int tok0 = (tile0 + j) * TS;
    // FULL (uniform): the page is present and all 16 tokens are inside the
    // context: no per-token masks (all pages of a row but its last)
    const bool full = ok && tok0 + TS <= Tb;
    // K and V images (V rows past the context or of a missing page: zeros,
    // so stale NaN / Inf cannot reach the MFMA; such K rows are masked)
    if (full) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        *reinterpret_cast<u32x4*>(kw + beam_lds_off(4 * c + lgrp, col)) = st.k[c];
        *reinterpret_cast<u32x4*>(vw + beam_lds_off(4 * c + lgrp, col)) = st.v[c];
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = 4 * c + lgrp;
        const bool vok = ok && tok0 + row < Tb;
        *reinterpret_cast<u32x4*>(kw + beam_lds_off(row, col)) = st.k[c];
        *reinterpret_cast<u32x4*>(vw + beam_lds_off(row, col)) =
            vok ? st.v[c] : u32x4{0u, 0u, 0u, 0u};
      }
    }
    // scores S[beam r][token] in lanes 0..15 (token = lane), register r:
    // A = q rows, B = K^T (token column col, dims 32 kk + 8 lgrp .. + 7)
    f32x4 sh = f32x4{0.f, 0.f, 0.f, 0.f}, sl = sh;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const f16x8 kf = __builtin_bit_cast(
          f16x8, *reinterpret_cast<const u32x4*>(kw + beam_lds_off(col, 4 * kk + lgrp)));
      sh = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[kk], kf, sh, 0, 0, 0);
      sl = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql[kk], kf, sl, 0, 0, 0);
    }
    // per-beam online softmax: the 16 tokens of beam r sit in one DPP row
    const bool tok_ok = lane < 16 && (full || (ok && tok0 + lane < Tb));
    float p[4], corr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool valid = tok_ok && ((mask >> r) & 1);
      const float sv = valid ? sh[r] + sl[r] * kLoUnscale : kNegSentinel;
      const float mnew = fmaxf(m4[r], row_max16(sv));
      corr[r] = __builtin_amdgcn_exp2f(m4[r] - mnew);
      p[r] = valid ? __builtin_amdgcn_exp2f(sv - mnew) : 0.f;
      l4[r] = l4[r] * corr[r] + group_sum<16>(p[r]);
      m4[r] = mnew;
    }
    if (lane < 16) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const _Float16 hi = p[r] >= kF16MinNormal ? (_Float16)p[r] : (_Float16)0.f;
        pw[r * 16 + lane] = hi;
        pw[(4 + r) * 16 + lane] = (_Float16)((p[r] - (float)hi) * kLoScale);
      }
    }
    // rescale the accumulators only when some beam's maximum moved (after the
    // first pages of a split, almost never): corr is exactly 1 otherwise
    if (__ballot(corr[0] != 1.f || corr[1] != 1.f || corr[2] != 1.f || corr[3] != 1.f)) {
      const float c0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(corr[0]), 0));
      const float c1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(corr[1]), 0));
      const float c2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(corr[2]), 0));
      const float c3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(corr[3]), 0));
      const int bcol = col & 3;
      const float cc = bcol == 0 ? c0 : bcol == 1 ? c1 : bcol == 2 ? c2 : c3;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] *= cc;
    }
    // P^T operand: beam column col, tokens 4 lgrp .. + 3
    const f16x4 pf = *reinterpret_cast<const f16x4*>(pw + col * 16 + 4 * lgrp);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // V^T operand of dims 16 i .. 16 i + 15: lane 4 qq + pp of group lgrp
      // addresses token row 4 lgrp + qq, dims 16 i + 4 pp .. + 3
      const int qq = col >> 2, pp = col & 3;
      const uint32_t ad = beam_lds_off(4 * lgrp + qq, 2 * i + (pp >> 1)) + 8 * (pp & 1);
      const s16x4 vt = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(vw + ad));
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, vt), pf, acc[i],
                                                      0, 0, 0);
    }
  };

  {
    Stage sa, sb;
    int i = it0;
    issue(sa, i);
    while (i < nitems) {
      issue(sb, i + istep);  // past the end: nothing loaded (num_records 0)
      process(sa, i);
      i += istep;
      if (i >= nitems) break;
      issue(sa, i + istep);
      process(sb, i);
      i += istep;
    }
  }

  // beam column b: fp16 part + residual part (columns b and b + 4)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[i][q] += __shfl_down(acc[i][q], 4, 16) * kLoUnscale;

  // combine the 4 waves' states per beam through LDS (each wave reuses its own
  // V image: acc [beam][128] then (m, l) [beam][2])
  float* red = reinterpret_cast<float*>(vw);
  if (col < 4) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[col * D + 16 * i + 4 * lgrp + q] = acc[i][q];
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[4 * D + 2 * r] = m4[r];
        red[4 * D + 2 * r + 1] = l4[r];
      }
    }
  }
  __syncthreads();
  if (brow) {
    float mv[4], M = kNegSentinel;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      mv[v] = reinterpret_cast<const float*>(vimg[v])[4 * D + 2 * w];
      M = fmaxf(M, mv[v]);
    }
    float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float* rv = reinterpret_cast<const float*>(vimg[v]);
      const float e = __builtin_amdgcn_exp2f(mv[v] - M);
      L += rv[4 * D + 2 * w + 1] * e;
      o0 += rv[w * D + 2 * lane] * e;
      o1 += rv[w * D + 2 * lane + 1] * e;
    }
    const size_t pidx = ((size_t)b * a.H + h) * a.nsplit + s;
    *reinterpret_cast<float2*>(a.part_acc + pidx * D + 2 * lane) = float2{o0, o1};
    if (lane == 0) {
      a.part_ml[pidx * 2] = M;
      a.part_ml[pidx * 2 + 1] = L;
    }
  }
}
#endif  // LLM_TUNING

// sum_s part[s * stride] * w_s over s < ns with w_s held by lane s (s < 64) /
// lane s - 64 of w1: loads issued 8 splits at a time so a merge costs a few
// memory round trips, not one per split; summation order s = 0, 1, ...
__device__ __forceinline__ float merge_splits(const float* part, int stride, int ns, float w0,
                                              float w1) {
  float acc = 0.f;
  for (int s0 = 0; s0 < ns; s0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (s0 + u < ns) ? part[(size_t)(s0 + u) * stride] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s2 = s0 + u;
      if (s2 < ns) {
        const float ws = s2 < 64 ? __shfl(w0, s2, 64) : __shfl(w1, s2 - 64, 64);
        acc += v[u] * ws;
      }
    }
  }
  return acc;
}

// Split merge (flash-decoding LSE combine): one wave per (b, h).
struct PaMergeArgs {
  const float* part_acc;
  const float* part_ml;
  float* out;
  const int32_t* context_lens;
  int B, H, D, T, TS, pps, nsplit, max_tiles;
};

__global__ __launch_bounds__(256) void pa_merge_kernel(PaMergeArgs a) {
  const int lane = lane_id();
  const int bh = blockIdx.x * 4 + wave_id_uniform();
  if (bh >= a.B * a.H) return;
  const int b = bh / a.H;
  int Tb = a.context_lens ? a.context_lens[b] : a.T;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + a.TS - 1) / a.TS, a.max_tiles);
  const int pps = row_pps(a.pps, a.nsplit, ntiles);
  // pps < 0: every split holds a partial (beam launches: cost-balanced splits)
  const int ns = a.pps < 0 ? a.nsplit : min(a.nsplit, (ntiles + pps - 1) / pps);
  const float* ml = a.part_ml + (size_t)bh * a.nsplit * 2;
  float M = kNegSentinel;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, ml[2 * s]);
  float* o = a.out + (size_t)bh * a.D;
  if (ns <= 0 || M <= 0.5f * kNegSentinel) {
    for (int d = lane; d < a.D; d += 64) o[d] = 0.f;
    return;
  }
  float L = 0.f;
  for (int s = 0; s < ns; ++s) L += ml[2 * s + 1] * __builtin_amdgcn_exp2f(ml[2 * s] - M);
  const float inv = 1.0f / (L + 1e-6f);
  const float* pa = a.part_acc + (size_t)bh * a.nsplit * a.D;
  const float w0 = lane < ns ? __builtin_amdgcn_exp2f(ml[2 * lane] - M) : 0.f;
  const float w1 = 64 + lane < ns ? __builtin_amdgcn_exp2f(ml[2 * (64 + lane)] - M) : 0.f;
  for (int d = lane; d < a.D; d += 64) o[d] = merge_splits(pa + d, a.D, ns, w0, w1) * inv;
}

// Split merge fused with the next consumer's input conversion: one workgroup
// per row b merges all H heads into an LDS row [H*D], then writes any of
//   out   fp32 [B][H*D]            (pa_decode's output)
//   q     int8 [B][H*D] + inv_scale[b]   (per-row quantisation of the o_proj
//         input, int8_quant.cpp:5-13,59-64 — replaces a quantize_rows launch)
//   out16 fp16 [B][H*D]            (fp16 o_proj input of the FP16 decoder)
struct PaMergeRowArgs {
  const float* part_acc;
  const float* part_ml;
  float* out;
  int8_t* q;
  float* inv_scale;
  _Float16* out16;
  const int32_t* context_lens;
  int B, H, D, T, TS, pps, nsplit, max_tiles;
  int pack;  // q / out16 in packed-A order (common.hpp a_frag_off_*)
  int ctx_p0;  // >= 0 and context_lens NULL: row b's context is ctx_p0 + b + 1 (prefill)
};

// DPL = output dims per lane (D / 64, at least 1).  A head's split weights
// (m, l) and the partials of its first kMergeBatch splits are loaded together,
// so a merge costs one memory round trip (splits beyond the batch: one more
// per batch); summation order s = 0, 1, ... as pa_merge_kernel.
constexpr int kMergeBatch = 8;

template <int DPL>
__global__ __launch_bounds__(1024) void pa_merge_row_kernel(PaMergeRowArgs a) {
  extern __shared__ float row[];  // [H*D]
  __shared__ float sh[16];
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int nw = blockDim.x >> 6;
  const int b = blockIdx.x;
  const int hid = a.H * a.D;
  int Tb = a.context_lens ? a.context_lens[b] : a.ctx_p0 >= 0 ? a.ctx_p0 + b + 1 : a.T;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + a.TS - 1) / a.TS, a.max_tiles);
  const int pps = row_pps(a.pps, a.nsplit, ntiles);
  // pps < 0: every split holds a partial (beam launches: cost-balanced splits)
  const int ns = a.pps < 0 ? a.nsplit : min(a.nsplit, (ntiles + pps - 1) / pps);
  for (int h = w; h < a.H; h += nw) {
    const size_t bh = (size_t)b * a.H + h;
    const float* ml = a.part_ml + bh * a.nsplit * 2;
    const float* pa = a.part_acc + bh * a.nsplit * a.D;
    // split weights, lane-parallel: lane holds splits lane and 64 + lane
    const float m0 = lane < ns ? ml[2 * lane] : kNegSentinel;
    const float m1 = 64 + lane < ns ? ml[2 * (64 + lane)] : kNegSentinel;
    const float l0 = lane < ns ? ml[2 * lane + 1] : 0.f;
    const float l1 = 64 + lane < ns ? ml[2 * (64 + lane) + 1] : 0.f;
    float v[kMergeBatch][DPL];
#pragma unroll
    for (int s2 = 0; s2 < kMergeBatch; ++s2)
#pragma unroll
      for (int j = 0; j < DPL; ++j) {
        const int d = lane + 64 * j;
        // unconditional loads (clamped in range) so all issue before the first wait
        v[s2][j] = pa[(size_t)min(s2, max(ns - 1, 0)) * a.D + min(d, a.D - 1)];
      }
    const float M = ln_wave_max(fmaxf(m0, m1));
    float* dst = row + h * a.D;
    if (ns <= 0 || M <= 0.5f * kNegSentinel) {
      for (int d = lane; d < a.D; d += 64) dst[d] = 0.f;
      continue;
    }
    const float w0 = lane < ns ? __builtin_amdgcn_exp2f(m0 - M) : 0.f;
    const float w1 = 64 + lane < ns ? __builtin_amdgcn_exp2f(m1 - M) : 0.f;
    // same summation order as pa_merge_kernel: s = 0, 1, ... (sequential);
    // split s's (l, w) come from lane s by readlane (SALU broadcast, no LDS
    // round trip per split), the first kMergeBatch unrolled
    float L = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < kMergeBatch; ++s2)
      if (s2 < ns) {
        const float ls = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l0), s2));
        const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));
        L += ls * ws;
      }
    for (int s2 = kMergeBatch; s2 < ns; ++s2) {
      const float ls = s2 < 64 ? __shfl(l0, s2, 64) : __shfl(l1, s2 - 64, 64);
      const float ws = s2 < 64 ? __shfl(w0, s2, 64) : __shfl(w1, s2 - 64, 64);
      L += ls * ws;
    }
    const float inv = 1.0f / (L + 1e-6f);
    float acc[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < kMergeBatch; ++s2) {
      const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));  // 0 past ns
#pragma unroll
      for (int j = 0; j < DPL; ++j) acc[j] += v[s2][j] * ws;
    }
    for (int s0 = kMergeBatch; s0 < ns; s0 += 8) {  // long splits lists (rare)
#pragma unroll
      for (int j = 0; j < DPL; ++j) {
        const int d = lane + 64 * j;
        float u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = (s0 + k < ns && d < a.D) ? pa[(size_t)(s0 + k) * a.D + d] : 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int s2 = s0 + k;
          if (s2 < ns) {
            const float ws = s2 < 64 ? __shfl(w0, s2, 64) : __shfl(w1, s2 - 64, 64);
            acc[j] += u[k] * ws;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
      const int d = lane + 64 * j;
      if (d < a.D) dst[d] = acc[j] * inv;
    }
  }
  __syncthreads();
  float am = 0.f;
  // packed int8 o_proj input only (the decode step): 4 values per thread, one
  // dword store each (4 consecutive k are 4 consecutive bytes of a fragment)
  const bool quad = a.q && a.pack && !a.out && !a.out16 && hid % 64 == 0;
  if (quad) {
    for (int i4 = threadIdx.x; i4 < hid / 4; i4 += blockDim.x) {
      const f32x4 v = reinterpret_cast<const f32x4*>(row)[i4];
      am = fmaxf(am, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
  } else {
    for (int i = threadIdx.x; i < hid; i += blockDim.x) {
      const float v = row[i];
      am = fmaxf(am, fabsf(v));
      if (a.out) a.out[(size_t)b * hid + i] = v;
      if (a.out16)
        a.out16[a.pack ? a_frag_off_f16(b, i, hid >> 5) : (size_t)b * hid + i] = (_Float16)v;
    }
  }
  if (!a.q) return;
  am = ln_wave_max(am);  // DPP (wave_max shuffles through LDS)
  if (lane == 0) sh[w] = am;
  __syncthreads();
  am = sh[0];
  for (int i = 1; i < nw; ++i) am = fmaxf(am, sh[i]);
  const float scale = 127.f / (am + 1e-6f);
  if (quad) {
    for (int i4 = threadIdx.x; i4 < hid / 4; i4 += blockDim.x)
      *reinterpret_cast<uint32_t*>(a.q + a_frag_off_i8(b, 4 * i4, hid >> 6)) =
          ln_quant4(reinterpret_cast<const f32x4*>(row)[i4], scale);
  } else {
    for (int i = threadIdx.x; i < hid; i += blockDim.x) {
      float y = roundf(__fmul_rn(row[i], scale));
      y = fminf(fmaxf(y, -128.f), 127.f);
      a.q[a.pack ? a_frag_off_i8(b, i, hid >> 6) : (size_t)b * hid + i] = (int8_t)(int)y;
    }
  }
  if (threadIdx.x == 0) a.inv_scale[b] = 1.0f / scale;
}

namespace {

constexpr int kMinPps = 8;
constexpr int kMaxWavesPerCu = 32;  // 8 per SIMD x 4 SIMDs (gfx950)

// Resident waves of the whole chip for one split-kernel instantiation
// (occupancy query x CU count), cached.  Fallback: 256 CUs x 3 waves/SIMD.
// Register stages of an instantiation: pages above 8 KiB hold a whole stage
// per page already (two would not fit the VGPR file).
template <int D, int TS, int KVT>
constexpr int split_stages() {
  return TS * D * kv_elem_bytes<KVT>() > 8192 ? 1 : 2;
}

template <int D, int TS, bool DIRECT, int KVT>
long long resident_waves() {
  static long long cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 0, blocks = 0;
  constexpr int ST = split_stages<D, TS, KVT>();
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &blocks, pa_split_kernel<D, TS, DIRECT, 16384, kKvLoadAux, ST, 0, false, false, KVT>, 256,
          0) == hipSuccess &&
      cus > 0 && blocks > 0) {
    cached = (long long)cus * blocks * 4;
  } else {
    (void)hipGetLastError();
    cached = 256LL * 4 * 3;
  }
  return cached;
}

// The MFMA beam-group kernel (D 128, page 16) exists only in the tuning build
// (LLM_BEAM_MFMA=1).  A private page costs it 4 items to a shared page's 1:
// split balance 64/16.
// The one-wave-per-beam-group kernel (pa_beam4_kernel) for row_group 4 fp16
// launches, tuning build only (LLM_BEAM4=1; LLM_BEAM4_SPLITS forces its split
// count): measured slower than the LDS-staged BEAM form of pa_split_kernel
// (C4 launch with merge: 69.2 us at 16 splits, 74.2 with two pages per
// register stage, 82.3 at 12 splits, against 67.6 us).
#ifndef BEAM4_MINW
#define BEAM4_MINW 2
#endif
#ifndef BEAM4_U
#define BEAM4_U 1
#endif
bool beam4_on() {
#if LLM_TUNING
  return env_int("LLM_BEAM4", 0) != 0;  // read per launch
#else
  return false;
#endif
}

#if LLM_TUNING
template <int D, int TS>
long long beam4_resident_waves() {
  if constexpr (TS * D * 2 > 8192) {
    return 0;
  } else {
  static long long cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 0, blocks = 0;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, pa_beam4_kernel<D, TS, BEAM4_MINW, BEAM4_U>, 256, 0) ==
          hipSuccess &&
      cus > 0 && blocks > 0) {
    cached = (long long)cus * blocks * 4;
  } else {
    (void)hipGetLastError();
    cached = 256LL * 4 * 3;
  }
  return cached;
  }
}

long long beam4_resident_for(int D, int TS) {
  auto by_ts = [&](auto d) -> long long {
    constexpr int DD = decltype(d)::value;
    return TS == 16 ? beam4_resident_waves<DD, 16>() : beam4_resident_waves<DD, 32>();
  };
  switch (D) {
    case 32: return by_ts(std::integral_constant<int, 32>{});
    case 64: return by_ts(std::integral_constant<int, 64>{});
    case 128: return by_ts(std::integral_constant<int, 128>{});
    default: return by_ts(std::integral_constant<int, 256>{});
  }
}
#else
long long beam4_resident_for(int, int) { return 0; }
#endif

bool beam_mfma_on() {
#if LLM_TUNING
  return env_int("LLM_BEAM_MFMA", 0) != 0;  // read per launch: a test sets and restores it
#else
  return false;
#endif
}
// Workgroup-merge form of the fp16 row-output launch (PaSplitArgs::wgm); the
// tuning build's LLM_WG_MERGE=0 restores split + merge launches (A/B, parity).
bool wg_merge_on() {
#if LLM_TUNING
  return env_int("LLM_WG_MERGE", 1) != 0;  // read per launch: a test flips it in-process
#else
  return true;
#endif
}
}  // namespace
// The FP16 decoder's o_proj fused into the workgroup merge (decoder.cpp
// oproj_fusable); the tuning build's LLM_OPROJ_FUSE=0 restores the o_proj
// GEMM launch (A/B, parity).
bool oproj_fuse_on() {
#if LLM_TUNING
  return env_int("LLM_OPROJ_FUSE", 1) != 0;
#else
  return true;
#endif
}
namespace {
int beam_mfma_balance16() {
#if LLM_TUNING
  static const int v = env_int("LLM_BEAM_MFMA_BALANCE16", 64);
  return v >= 16 ? v : 0;
#else
  return 64;
#endif
}

template <int D, int TS, int KVT>
hipError_t launch_split(const PaSplitArgs& a, bool direct, hipStream_t st, bool* beam) {
  const int waves = ((a.B + a.group - 1) / a.group) * a.group * a.H * a.nsplit;
  const dim3 grid((waves + 3) / 4), block(256);
  if constexpr (KVT != LLM_F16) {
    // other KV element types: the standard schedule (no beam-prefetch form)
    constexpr int ST = split_stages<D, TS, KVT>();
    if (direct)
      hipLaunchKernelGGL((pa_split_kernel<D, TS, true, 16384, kKvLoadAux, ST, 0, false, false, KVT>),
                         grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((pa_split_kernel<D, TS, false, 16384, kKvLoadAux, ST, 0, false, false, KVT>),
                         grid, block, 0, st, a);
    return hipGetLastError();
  }
  constexpr int ST = split_stages<D, TS, LLM_F16>();
  if (a.wgm) {  // pa_decode_internal: group 1, 2..8 splits, not direct
    if constexpr (D <= kOprojMaxD) {
      if (a.o_acc) {
        hipLaunchKernelGGL((pa_split_kernel<D, TS, false, 16384, kKvLoadAux, ST, 0, false, false,
                                            LLM_F16, true, true, true>),
                           dim3(a.B * a.H), dim3(64 * a.nsplit), 0, st, a);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((pa_split_kernel<D, TS, false, 16384, kKvLoadAux, ST, 0, false, false,
                                        LLM_F16, true, true>),
                       dim3(a.B * a.H), dim3(64 * a.nsplit), 0, st, a);
    return hipGetLastError();
  }
#if LLM_TUNING
  if (a.group == 4 && !direct && ST == 2 && a.beam4) {
    // pa_beam4_kernel: one wave per (group, head, split)
    const int waves4 = ((a.B + 3) / 4) * a.H * a.nsplit;
    if constexpr (TS * D * 2 <= 8192)
      hipLaunchKernelGGL((pa_beam4_kernel<D, TS, BEAM4_MINW, BEAM4_U>), dim3((waves4 + 3) / 4), dim3(256), 0,
                         st, a);
    *beam = true;
    return hipGetLastError();
  }
#endif
  if (a.group == 4 && !direct && ST == 2) {
    // 8 KiB register stages: 112 VGPRs, 4 waves per SIMD.  The 16 KiB form
    // (179 VGPRs, 2 waves) spent 27 % of its wave time in issue stalls and
    // 20 % parked (SQ PMC, scripts/gpu_sq_pmc.sh); same-box A/B of the C4
    // launch: 72-74 vs 76 us (scripts/ab_attention_lib.py, -DLLM_BEAM_CHUNK=)
#ifndef LLM_BEAM_CHUNK
#define LLM_BEAM_CHUNK 8192
#define LLM_BEAM_WAVES 0
#endif
#if LLM_TUNING
    if constexpr (D == 128 && TS == 16) {
      if (beam_mfma_on()) {
        PaSplitArgs am = a;
        am.balance16 = beam_mfma_balance16();
        static const int dbg = env_int("LLM_BEAM_MFMA_DBG", 0);
        if (dbg == 1)
          hipLaunchKernelGGL(pa_beam_mfma_kernel<1>, grid, block, 0, st, am);
        else if (dbg == 2)
          hipLaunchKernelGGL(pa_beam_mfma_kernel<2>, grid, block, 0, st, am);
        else
        hipLaunchKernelGGL(pa_beam_mfma_kernel<0>, grid, block, 0, st, am);
        *beam = true;
        return hipGetLastError();
      }
    }
#endif
    hipLaunchKernelGGL((pa_split_kernel<D, TS, false, LLM_BEAM_CHUNK, kKvLoadAux, 2, LLM_BEAM_WAVES,
                                        false, true>), grid, block, 0, st, a);
    *beam = true;
  } else if (direct) {
    hipLaunchKernelGGL((pa_split_kernel<D, TS, true, 16384, kKvLoadAux, ST>), grid, block, 0, st, a);
  } else {
    hipLaunchKernelGGL((pa_split_kernel<D, TS, false, 16384, kKvLoadAux, ST>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

template <int D, int KVT>
hipError_t dispatch_ts(const PaSplitArgs& a, int TS, bool direct, hipStream_t st, bool* beam) {
  constexpr int ES = kv_elem_bytes<KVT>();
  if (TS == 16) {
    if constexpr (kv_shape_ok(D, 16, ES)) return launch_split<D, 16, KVT>(a, direct, st, beam);
  } else if (TS == 32) {
    if constexpr (kv_shape_ok(D, 32, ES)) return launch_split<D, 32, KVT>(a, direct, st, beam);
  }
  return hipErrorInvalidValue;
}

template <int D>
hipError_t dispatch_kvt(const PaSplitArgs& a, int kvt, int TS, bool direct, hipStream_t st,
                        bool* beam) {
  switch (kvt) {
    case LLM_F16: return dispatch_ts<D, LLM_F16>(a, TS, direct, st, beam);
    case LLM_BF16: return dispatch_ts<D, LLM_BF16>(a, TS, direct, st, beam);
    case LLM_F32: return dispatch_ts<D, LLM_F32>(a, TS, direct, st, beam);
    case LLM_I8: return dispatch_ts<D, LLM_I8>(a, TS, direct, st, beam);
    default: return hipErrorInvalidValue;
  }
}

int kv_dtype_bytes(int kvt) {
  switch (kvt) {
    case LLM_F16: case LLM_BF16: return 2;
    case LLM_F32: return 4;
    case LLM_I8: return 1;
    default: return 0;
  }
}

bool supported(int D, int TS, int kvt) {
  const int es = kv_dtype_bytes(kvt);
  return es > 0 && (D == 32 || D == 64 || D == 128 || D == 256) && (TS == 16 || TS == 32) &&
         kv_shape_ok(D, TS, es);
}

// Upper bound of the split count of any launch over rows of <= ntiles tiles
// (workspace sizing; host-only, no device query).
long long max_nsplit(int B, int H, int ntiles) {
  ntiles = std::max(ntiles, 1);
  const long long bh = std::max(1LL, (long long)B * H);
  const long long cap = 256LL * kMaxWavesPerCu;  // largest resident-wave count
  const long long lo = (ntiles + kMaxPps - 1) / kMaxPps;
  return std::min<long long>(
      kMaxSplits,
      std::max(lo, std::min<long long>((ntiles + kMinPps - 1) / kMinPps, lo + (cap + bh - 1) / bh + 1)));
}

// Splits per (b, h): the smallest NS that is a whole number of resident-wave
// rounds (B*H*NS ~ k * resident) with splits of <= kMaxPps pages, so every wave
// carries the same page count and the last round is not a ragged tail; never
// below kMinPps pages per split.  Small launches, where a full round would
// leave each wave under kShortPps pages, use fewer, longer splits instead,
// as long as at least kMinLaunchWaves waves remain: a split's fixed cost
// (page ids, q, its partial and its share of the merge) outweighs an idle
// part of the chip there.  Measured (scripts/sweep_attention_pps.py), round
// rule -> this rule: C2 (16 x 12 heads, 2048 tokens) 25.1 -> 21.3 us;
// 64 x 12 x 2048: 72.7 -> 66.6 us; 8 x 16 x 4096: 49.3 -> 46.1 us;
// 1 x 16 x 8192: 32.8 -> 26.4 us; 4 x 12 x 1024 unchanged (9.9 us).
constexpr int kShortPps = 32;
constexpr long long kMinLaunchWaves = 512;
// Workgroup-merge launches (PaSplitArgs::wgm) have no merge launch to feed, so
// their splits stay long: C2 (130 tiles) 3 splits, not 5.  Same-box C2 sweep
// (scripts/gpu_wgm_splits.sh, forced splits 2 / 3 / 4 / 5 / 6 / 8):
// 27.4-28.0k / 29.6-30.1k / 29.1-29.2k / 28.4k / 28.6-28.9k / 28.2-29.0k tok/s.
constexpr int kWgmShortPps = 64;
int choose_nsplit(int B, int H, int ntiles, int pps_fixed, long long resident,
                  int short_pps = kShortPps) {
  ntiles = std::max(ntiles, 1);
  if (pps_fixed > 0) {
    const int pps = std::min(pps_fixed, kMaxPps);
    return (ntiles + pps - 1) / pps;
  }
  const long long bh = std::max(1LL, (long long)B * H);
  const long long lo = (ntiles + kMaxPps - 1) / kMaxPps;
  long long ns = lo;
  for (long long k = 1; k <= 64; ++k) {
    const long long cand = (k * resident + bh - 1) / bh;
    if (cand >= lo) { ns = cand; break; }
  }
  ns = std::min<long long>(ns, std::max(1, (ntiles + kMinPps - 1) / kMinPps));
  if ((ntiles + ns - 1) / ns < short_pps)
    ns = std::min(ns, std::max<long long>((ntiles + short_pps - 1) / short_pps,
                                          (kMinLaunchWaves + bh - 1) / bh));
  ns = std::max(ns, lo);
  return (int)std::min(ns, max_nsplit(B, H, ntiles));
}

template <int D, int TS, int KVT>
long long resident_for() {
  if constexpr (kv_shape_ok(D, TS, kv_elem_bytes<KVT>()))
    return resident_waves<D, TS, false, KVT>();
  return 256LL * 4 * 3;
}

template <int D>
long long resident_for_kvt(int TS, int kvt) {
  auto by_ts = [&](auto k) -> long long {
    constexpr int K = decltype(k)::value;
    return TS == 16 ? resident_for<D, 16, K>() : resident_for<D, 32, K>();
  };
  switch (kvt) {
    case LLM_BF16: return by_ts(std::integral_constant<int, LLM_BF16>{});
    case LLM_F32: return by_ts(std::integral_constant<int, LLM_F32>{});
    case LLM_I8: return by_ts(std::integral_constant<int, LLM_I8>{});
    default: return by_ts(std::integral_constant<int, LLM_F16>{});
  }
}

long long resident_waves_for(int D, int TS, int kvt) {
  auto pick = [&](auto d) -> long long {
    constexpr int DD = decltype(d)::value;
    return resident_for_kvt<DD>(TS, kvt);
  };
  switch (D) {
    case 32: return pick(std::integral_constant<int, 32>{});
    case 64: return pick(std::integral_constant<int, 64>{});
    case 128: return pick(std::integral_constant<int, 128>{});
    default: return pick(std::integral_constant<int, 256>{});
  }
}

}  // namespace

int pa_pages_per_split(int B, int H, int T, int TS, int max_tiles) {
  const int ntiles = std::max(1, std::min((T + TS - 1) / TS, max_tiles));
  const int ns = choose_nsplit(B, H, ntiles, 0, 256LL * 4 * 3);
  return (ntiles + ns - 1) / ns;
}

}  // namespace llm

using namespace llm;

extern "C" int pa_decode_pages_per_split(int B, int H, int T, int page_size, int max_tiles) {
  if (B < 0 || H <= 0 || T < 0 || page_size <= 0 || max_tiles <= 0) return -1;
  return pa_pages_per_split(B, H, T, page_size, max_tiles);
}

extern "C" size_t pa_decode_workspace_bytes(int B, int H, int D, int max_tiles,
                                            int pages_per_split) {
  if (B <= 0 || H <= 0 || D <= 0 || max_tiles <= 0) return 0;
  const size_t nsplit = pages_per_split > 0
                            ? (size_t)choose_nsplit(B, H, max_tiles, pages_per_split, 0)
                            : (size_t)max_nsplit(B, H, max_tiles);
  return (size_t)B * H * nsplit * (size_t)(D + 2) * sizeof(float);
}

int llm::pa_merge_splits_internal(const float* part_acc, const float* part_ml, float* out,
                                  const int32_t* context_lens, int B, int H, int D, int T, int TS,
                                  int pps, int nsplit, int max_tiles, hipStream_t st) {
  PaMergeArgs mg{part_acc, part_ml, out, context_lens, B, H, D, T, TS, pps, nsplit, max_tiles};
  hipLaunchKernelGGL(pa_merge_kernel, dim3((B * H + 3) / 4), dim3(256), 0, st, mg);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}

int llm::pa_merge_rows_internal(const float* part_acc, const float* part_ml, float* out,
                                const PaRowOutputs* rows, const int32_t* context_lens, int ctx_p0,
                                int B, int H, int D, int T, int TS, int pps, int nsplit,
                                int max_tiles, hipStream_t st) {
  PaMergeRowArgs mg{part_acc, part_ml, out, rows ? rows->q : nullptr,
                    rows ? rows->inv_scale : nullptr,
                    rows ? static_cast<_Float16*>(rows->out16) : nullptr, context_lens, B, H, D, T,
                    TS, pps, nsplit, max_tiles, rows ? rows->pack : 0, ctx_p0};
  const int threads = 64 * std::min(16, H);  // one wave per head (heads > 16 loop)
  const size_t lds = (size_t)H * D * sizeof(float);
  if (D <= 64)
    hipLaunchKernelGGL(pa_merge_row_kernel<1>, dim3(B), dim3(threads), lds, st, mg);
  else if (D <= 128)
    hipLaunchKernelGGL(pa_merge_row_kernel<2>, dim3(B), dim3(threads), lds, st, mg);
  else
    hipLaunchKernelGGL(pa_merge_row_kernel<4>, dim3(B), dim3(threads), lds, st, mg);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}

namespace {
// Cost of a beam-private tile relative to a shared one, in 1/16ths (beam-group
// launches, dynamic splits).  In the tuning build (make tune) LLM_BEAM_BALANCE16
// overrides it (0: equal tile counts, the plain partition).
int beam_balance16() {
#if LLM_TUNING
  static const int v = [] {
    const char* e = std::getenv("LLM_BEAM_BALANCE16");
    const int x = e ? std::atoi(e) : 44;
    return x >= 16 ? x : 0;
  }();
  return v;
#else
  return 44;  // measured sweep in DESIGN.md §8 (C4 launch 84 -> 66 us)
#endif
}

template <int D, int TS>
hipError_t beam_occupancy(int* blocks) {
#if LLM_TUNING
  if (D == 128 && TS == 16 && beam_mfma_on())
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, pa_beam_mfma_kernel<0>, 256, 0);
#endif
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(
      blocks, pa_split_kernel<D, TS, false, LLM_BEAM_CHUNK, kKvLoadAux, 2, LLM_BEAM_WAVES, false, true>,
      256, 0);
}

// Resident waves of the beam-group kernel (0 where the plain schedule runs
// instead: pages above 8 KiB).
template <int D, int TS>
long long beam_resident_waves() {
  if constexpr (!kv_shape_ok(D, TS, 2) || split_stages<D, TS, LLM_F16>() != 2) {
    return 0;
  } else {
    static long long cached = -1;
    if (cached >= 0) return cached;
    int dev = 0, cus = 0, blocks = 0;
    cached = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        beam_occupancy<D, TS>(&blocks) == hipSuccess &&
        cus > 0 && blocks > 0)
      cached = (long long)cus * blocks * 4;
    else
      (void)hipGetLastError();
    return cached;
  }
}

long long beam_resident_waves_for(int D, int TS) {
  auto by_ts = [&](auto d) -> long long {
    constexpr int DD = decltype(d)::value;
    return TS == 16 ? beam_resident_waves<DD, 16>() : beam_resident_waves<DD, 32>();
  };
  switch (D) {
    case 32: return by_ts(std::integral_constant<int, 32>{});
    case 64: return by_ts(std::integral_constant<int, 64>{});
    case 128: return by_ts(std::integral_constant<int, 128>{});
    default: return by_ts(std::integral_constant<int, 256>{});
  }
}
}  // namespace

int llm::pa_decode_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                            const int32_t* beam_ids, const int32_t* context_lens, int B, int H,
                            int D, int T, float sm_scale, int pages_per_split, void* workspace,
                            size_t workspace_bytes, hipStream_t st, const PaRowOutputs* rows,
                            int row_group, PaPlan* plan) {
  LLM_REQUIRE(kv != nullptr, "pa_decode: kv view is NULL");
  LLM_REQUIRE(B >= 0 && H > 0 && D > 0 && T >= 0, "pa_decode: bad B/H/D/T");
  if (plan) *plan = PaPlan{};
  if (B == 0) return LLM_OK;
  const bool row_out = rows && (rows->q || rows->out16);
  // the FP16 decoder's fused o_proj (PaRowOutputs::o_acc): workgroup-merge launches only
  const bool oproj = rows && rows->o_acc && !rows->q && !rows->f32_rows;
  LLM_REQUIRE(plan || (q != nullptr && (out != nullptr || row_out || oproj)), "pa_decode: q/out NULL");
  LLM_REQUIRE(!oproj || (rows->wo_heads && rows->o_x && rows->o_flag && rows->o_n > 0 &&
                         D <= kOprojMaxD && H <= 64),
              "pa_decode: fused o_proj needs W_o head slices, an output, a range flag, o_n > 0, "
              "head_dim <= 128 and at most 64 heads");
  LLM_REQUIRE(!rows || !rows->q || rows->inv_scale, "pa_decode: row quantisation needs inv_scale");
  LLM_REQUIRE(!row_out || (size_t)H * D * 4 <= 65536, "pa_decode: row outputs need H*D <= 16384");
  LLM_REQUIRE(!rows || !rows->pack || (H * D) % 64 == 0, "pa_decode: packed row outputs need H*D % 64 == 0");
  LLM_REQUIRE(kv->k_pool && kv->v_pool && kv->page_table, "pa_decode: kv pointers NULL");
  LLM_REQUIRE(kv_dtype_bytes(kv->kv_dtype) > 0,
              "pa_decode: kv_dtype must be LLM_F16, LLM_BF16, LLM_F32 or LLM_I8");
  LLM_REQUIRE(kv->num_heads == H, "pa_decode: H != kv->num_heads");
  LLM_REQUIRE(kv->head_dim == D, "pa_decode: D != kv->head_dim");
  LLM_REQUIRE(kv->num_pages > 0 && kv->num_beams > 0 && kv->max_tiles > 0,
              "pa_decode: empty kv view");
  if (!supported(D, kv->page_size, kv->kv_dtype))
    return fail(LLM_ERR_UNSUPPORTED, "pa_decode: unsupported head_dim/page_size/kv_dtype (D in "
                                     "{32,64,128,256}, page_size in {16,32}, one page of "
                                     "1..16 KiB)");
  const size_t page_stride = kv_view_page_stride(*kv);
  LLM_REQUIRE(page_stride >= (size_t)kv->page_size * D * kv_dtype_bytes(kv->kv_dtype) &&
                  page_stride % 16 == 0,
              "pa_decode: page_stride must be 0 or >= one page and a multiple of 16");
  LLM_REQUIRE((long long)kv->num_pages * (long long)page_stride < (1LL << 47),
              "pa_decode: pool too large");
  const int TS = kv->page_size;
  // tiles at or past max_tiles have no page-table entry: they are missing (masked)
  const int ntiles_max = std::max(1, std::min((T + TS - 1) / TS, kv->max_tiles));
  const int pps_fixed = pages_per_split > 0 ? std::min(pages_per_split, kMaxPps) : 0;
  const long long resident = pps_fixed <= 0 ? resident_waves_for(D, TS, kv->kv_dtype) : 0;
  // beam-group launches size their splits for the beam kernel's occupancy
  // (4 waves per SIMD against the plain kernel's 2: C4 8 splits, not 4)
  const long long resident_launch =
      pps_fixed <= 0 && row_group == 4 && kv->kv_dtype == LLM_F16
          ? std::max(resident, beam_resident_waves_for(D, TS)) : resident;
  // fp16 o_proj input only (the FP16 decoder's attention): with at most one
  // merge batch of splits per (b, h) the splits merge inside the split
  // launch's workgroup (C2: 12 merge launches per step fewer), with long splits
  // fp32 rows for a quantising consumer (the INT8 decoder's o_proj prologue)
  // merge in the workgroup too, with a split count that divides the CU's 8
  // resident waves (2 / 4 / 8 waves per workgroup: a 6-wave workgroup would
  // leave 2 of the 8 slots idle): C3 6 -> 8 splits
  const bool f32_rows = rows && rows->f32_rows && !rows->q && !rows->out16;
  const bool wgm_ok = ((row_out && rows->out16 && !rows->q) || oproj || f32_rows) && row_group == 1 &&
                      kv->kv_dtype == LLM_F16 && wg_merge_on();
  int nsplit = choose_nsplit(B, H, ntiles_max, pps_fixed, resident_launch);
  if (wgm_ok && pps_fixed <= 0 && !f32_rows) {
    const int nw = choose_nsplit(B, H, ntiles_max, 0, resident_launch, kWgmShortPps);
    if (nw >= 2 && nw <= kWgmMaxSplits) nsplit = nw;
  }
  if (wgm_ok && pps_fixed <= 0 && f32_rows && nsplit >= 2) {
    int nw = 2;
    while (nw < nsplit && nw < kWgmMaxSplits) nw *= 2;
    if (nw >= nsplit && (long long)nw * kMaxPps >= ntiles_max) nsplit = nw;
  }
#if LLM_TUNING
  // tuning build: LLM_WGM_SPLITS forces the split count of workgroup-merge
  // eligible launches (fp16 row outputs, dynamic splits)
  if (rows && (rows->out16 || oproj) && !rows->q && row_group == 1 && pps_fixed <= 0) {
    const int f = env_int("LLM_WGM_SPLITS", 0);
    if (f >= 2 && f <= kWgmMaxSplits && (long long)f * kMaxPps >= ntiles_max) nsplit = f;
  }
#endif
  // beam groups of 4 rows (fp16 pages <= 8 KiB, dynamic splits): pa_beam4_kernel,
  // one wave per (group, head, split), splits sized for its own occupancy (a
  // whole number of resident rounds over (group, head) pairs), each split
  // holding <= 128 page items; fixed pages_per_split keeps the BEAM form
  bool use_beam4 = false;
  if (row_group == 4 && pps_fixed <= 0 && kv->kv_dtype == LLM_F16 && TS * D * 2 <= 8192 &&
      beam4_on() && !beam_mfma_on()) {
    const long long groups = (long long)((B + 3) / 4) * H;
    const long long need = (4LL * ntiles_max + kMaxPps - 1) / kMaxPps;
    long long ns = (beam4_resident_for(D, TS) + groups - 1) / groups;
    ns = std::max(std::max(ns, need), 2LL);
    ns = std::min(ns, max_nsplit(B, H, ntiles_max));
#if LLM_TUNING
    const int f = env_int("LLM_BEAM4_SPLITS", 0);
    if (f >= 2) ns = std::min<long long>(f, max_nsplit(B, H, ntiles_max));
#endif
    if (ns >= need && ns >= 2) {
      use_beam4 = true;
      nsplit = (int)ns;
    }
  }
  if (nsplit > kMaxSplits || (long long)nsplit * (pps_fixed > 0 ? pps_fixed : kMaxPps) < ntiles_max)
    return fail(LLM_ERR_UNSUPPORTED,
                "pa_decode: at most 128 splits of at most 128 pages per row (raise "
                "pages_per_split, or pass 0; T <= 16384 pages)");
  const bool direct = nsplit <= 1;
  if (plan) {
    const int group = std::max(1, std::min(row_group, 4));
    const bool wg = wgm_ok && !direct && group == 1 && nsplit <= kWgmMaxSplits;
    const bool beam = group == 4 && !direct && kv->kv_dtype == LLM_F16 &&
                      TS * D * 2 <= 8192;
    plan->nsplit = nsplit;
    plan->form = (direct ? LLM_PA_FORM_DIRECT : wg ? LLM_PA_FORM_WG_MERGE
                  : row_out ? LLM_PA_FORM_SPLIT_MERGE_ROW : LLM_PA_FORM_SPLIT_MERGE) |
                 (beam ? LLM_PA_FORM_BEAM : 0) | (oproj && wg ? LLM_PA_FORM_OPROJ : 0);
    return LLM_OK;
  }
  LLM_REQUIRE(!direct || out != nullptr, "pa_decode: single-split launch needs the fp32 out");
  if (oproj && (direct || row_group != 1 || nsplit > kWgmMaxSplits || !wgm_ok))
    return fail(LLM_ERR_UNSUPPORTED, "pa_decode: the fused o_proj needs the workgroup-merge form");

  PaSplitArgs a{};
  a.k_pool = static_cast<const uint8_t*>(kv->k_pool);
  a.v_pool = static_cast<const uint8_t*>(kv->v_pool);
  a.page_table = kv->page_table;
  a.q = q;
  a.q_stride = q_stride;
  a.out = out;
  a.beam_ids = beam_ids;
  a.context_lens = context_lens;
  a.B = B;
  a.H = H;
  a.T = T;
  a.num_pages = kv->num_pages;
  a.num_beams = kv->num_beams;
  a.max_tiles = kv->max_tiles;
  a.page_stride = page_stride;
  a.pps = pps_fixed;
  a.nsplit = nsplit;
  a.group = std::max(1, std::min(row_group, 4));
  a.qscale = sm_scale * kLog2e;
  const bool wgm = wgm_ok && !direct && a.group == 1 && nsplit <= kWgmMaxSplits;
  if (!direct && !wgm) {  // (the workgroup merge keeps its splits' states in LDS)
    const size_t need = (size_t)B * H * nsplit * (size_t)(D + 2) * sizeof(float);
    LLM_REQUIRE(workspace != nullptr && workspace_bytes >= need,
                "pa_decode: workspace too small (see pa_decode_workspace_bytes)");
    a.part_acc = static_cast<float*>(workspace);
    a.part_ml = a.part_acc + (size_t)B * H * nsplit * D;
  }
  a.balance16 = beam_balance16();
  a.beam4 = use_beam4 ? 1 : 0;
  if (wgm) {
    a.wgm = 1;
    a.out16 = static_cast<_Float16*>(rows->out16);
    a.pack = rows->pack;
    a.out = rows->keep_out || f32_rows ? out : nullptr;
    if (oproj) {
      a.o_acc = rows->o_acc;
      a.o_x = rows->o_x;
      a.wo_heads = static_cast<const _Float16*>(rows->wo_heads);
      a.o_n = rows->o_n;
      a.o_flag = rows->o_flag;
    }
  }
  hipError_t e;
  bool beam = false;  // the beam kernel ran: every split holds a partial
  switch (D) {
    case 32: e = dispatch_kvt<32>(a, kv->kv_dtype, TS, direct, st, &beam); break;
    case 64: e = dispatch_kvt<64>(a, kv->kv_dtype, TS, direct, st, &beam); break;
    case 128: e = dispatch_kvt<128>(a, kv->kv_dtype, TS, direct, st, &beam); break;
    default: e = dispatch_kvt<256>(a, kv->kv_dtype, TS, direct, st, &beam); break;
  }
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("pa_split launch: ") + hipGetErrorString(e));
  if (wgm) return LLM_OK;
  if (row_out && !direct)
    return pa_merge_rows_internal(a.part_acc, a.part_ml, rows->keep_out ? out : nullptr, rows,
                                  context_lens, -1, B, H, D, T, TS, beam ? -1 : pps_fixed, nsplit,
                                  kv->max_tiles, st);
  if (!direct) {
    const int r = pa_merge_splits_internal(a.part_acc, a.part_ml, out, context_lens, B, H, D, T,
                                           TS, beam ? -1 : pps_fixed, nsplit, kv->max_tiles, st);
    if (r != LLM_OK) return r;
  }
  if (row_out) {  // single split: out is final; convert it in a row pass
    if (rows->q)
      LLM_HIP_RET(launch_quantize_rows(out, B, H * D, rows->q, rows->inv_scale, st, rows->pack));
    if (rows->out16)
      LLM_HIP_RET(launch_to_f16(out, (size_t)B * H * D, rows->out16, st, rows->pack ? H * D : 0));
  }
  return LLM_OK;
}

extern "C" int pa_decode_grouped(const pa_kv_view* kv, const float* q, float* out,
                                 const int32_t* beam_ids, const int32_t* context_lens, int B,
                                 int H, int D, int T, float sm_scale, int pages_per_split,
                                 int row_group, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  LLM_REQUIRE(row_group >= 1 && row_group <= 4, "pa_decode_grouped: row_group must be in [1, 4]");
  return pa_decode_internal(kv, q, H * D, out, beam_ids, context_lens, B, H, D, T, sm_scale,
                            pages_per_split, workspace, workspace_bytes, as_stream(stream),
                            nullptr, row_group);
}

extern "C" int pa_decode_plan(const pa_kv_view* kv, int B, int H, int D, int T,
                              int pages_per_split, int row_group, int* nsplit, int* form) {
  LLM_REQUIRE(nsplit && form, "pa_decode_plan: NULL output");
  LLM_REQUIRE(row_group >= 1 && row_group <= 4, "pa_decode_plan: row_group must be in [1, 4]");
  PaPlan p;
  const int rc = pa_decode_internal(kv, nullptr, H * D, nullptr, nullptr, nullptr, B, H, D, T, 1.f,
                                    pages_per_split, nullptr, 0, nullptr, nullptr, row_group, &p);
  *nsplit = p.nsplit;
  *form = p.form;
  return rc;
}

extern "C" int pa_decode(const pa_kv_view* kv, const float* q, float* out,
                         const int32_t* beam_ids, const int32_t* context_lens, int B, int H,
                         int D, int T, float sm_scale, int pages_per_split, void* workspace,
                         size_t workspace_bytes, void* stream) {
  return pa_decode_internal(kv, q, H * D, out, beam_ids, context_lens, B, H, D, T, sm_scale,
                            pages_per_split, workspace, workspace_bytes, as_stream(stream));
}

#if LLM_TUNING
// Tuning hook (not part of include/llm_decoder.h): run the split kernel of
// D=128 / TS=16 in a given variant so scripts/bench_kernels.py can compare
// register-stage sizes and cache policies in one process.
extern "C" int pa_decode_tune(int variant, const pa_kv_view* kv, const float* q, float* out,
                              const int32_t* context_lens, int B, int H, int T, int pps,
                              void* workspace, size_t workspace_bytes, void* stream) {
  LLM_REQUIRE(kv && (kv->head_dim == 128 || kv->head_dim == 64) && kv->page_size == 16 &&
                  H == kv->num_heads,
              "pa_decode_tune: D 128 (variants 0-19) or 64 (20-25), page 16 only");
  const int D = kv->head_dim;
  LLM_REQUIRE((D == 128) == (variant < 20), "pa_decode_tune: variant / head_dim mismatch");
  const int ntiles_max = std::max(1, (T + 15) / 16);
  pps = std::min(std::max(pps, 1), kMaxPps);
  const int nsplit = (ntiles_max + pps - 1) / pps;
  LLM_REQUIRE(nsplit > 1 && nsplit <= kMaxSplits, "pa_decode_tune: needs 2..128 splits");
  const size_t need = (size_t)B * H * nsplit * (D + 2) * sizeof(float);
  LLM_REQUIRE(workspace && workspace_bytes >= need, "pa_decode_tune: workspace");
  PaSplitArgs a{};
  a.k_pool = static_cast<const uint8_t*>(kv->k_pool);
  a.v_pool = static_cast<const uint8_t*>(kv->v_pool);
  a.page_table = kv->page_table;
  a.q = q; a.q_stride = H * D; a.out = out;
  a.context_lens = context_lens;
  a.B = B; a.H = H; a.T = T;
  a.num_pages = kv->num_pages; a.num_beams = kv->num_beams; a.max_tiles = kv->max_tiles;
  a.page_stride = kv_view_page_stride(*kv);
  a.pps = pps; a.nsplit = nsplit; a.group = 1; a.qscale = kLog2e;
  a.part_acc = static_cast<float*>(workspace);
  a.part_ml = a.part_acc + (size_t)B * H * nsplit * D;
  hipStream_t st = as_stream(stream);
  const dim3 grid((B * H * nsplit + 3) / 4), block(256);
  switch (variant) {  // NOLINT
    case 0: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 0>), grid, block, 0, st, a); break;
    case 1: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 2>), grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 0>), grid, block, 0, st, a); break;
    case 3: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 2>), grid, block, 0, st, a); break;
    case 4: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 32768, 0>), grid, block, 0, st, a); break;
    case 5: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 32768, 2>), grid, block, 0, st, a); break;
    case 6: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 2, 1, 8>), grid, block, 0, st, a); break;
    case 7: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 2, 1, 4>), grid, block, 0, st, a); break;
    case 8: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 2, 2, 4>), grid, block, 0, st, a); break;
    case 9: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 2, 1, 6>), grid, block, 0, st, a); break;
    case 10: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 2, 2, 0, true>), grid, block, 0, st, a); break;
    case 11: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, 2, 1, 8, true>), grid, block, 0, st, a); break;
    case 12: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 32768, 2, 2, 0, true>), grid, block, 0, st, a); break;
    // 13: variant 1 without the full-page fast path (every token takes the validity selects)
    case 13: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 2, 2, 0, false, false, LLM_F16, false>), grid, block, 0, st, a); break;
    // 14-18: variant 1 with other cache-policy bits of the KV loads (gfx940-family
    // CPol: sc0 = 1, nt = 2, sc1 = 16): 14 sc0|nt, 15 sc1|nt, 16 sc0|sc1|nt,
    // 17 sc1, 18 sc0; 19: loads only with sc1|nt
    case 14: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 3>), grid, block, 0, st, a); break;
    case 15: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 18>), grid, block, 0, st, a); break;
    case 16: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 19>), grid, block, 0, st, a); break;
    case 17: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 16>), grid, block, 0, st, a); break;
    case 18: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 1>), grid, block, 0, st, a); break;
    case 19: hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 16384, 18, 2, 0, true>), grid, block, 0, st, a); break;
    // D = 64 (C2): 20 production, 21 one 16 KiB stage, 22 8 KiB stages, 23 one
    // 32 KiB stage, 24 / 25 loads only (16 KiB x 2, 32 KiB x 1)
    case 20: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 16384, 2, 2>), grid, block, 0, st, a); break;
    case 21: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 16384, 2, 1>), grid, block, 0, st, a); break;
    case 22: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 8192, 2, 2>), grid, block, 0, st, a); break;
    case 23: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 32768, 2, 1>), grid, block, 0, st, a); break;
    case 24: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 16384, 2, 2, 0, true>), grid, block, 0, st, a); break;
    case 25: hipLaunchKernelGGL((pa_split_kernel<64, 16, false, 32768, 2, 1, 0, true>), grid, block, 0, st, a); break;
    default: return fail(LLM_ERR_INVALID, "pa_decode_tune: variant");
  }
  LLM_HIP_RET(hipGetLastError());
  PaMergeArgs mg{a.part_acc, a.part_ml, out, context_lens, B, H, D, T, 16, pps, nsplit,
                 kv->max_tiles};
  hipLaunchKernelGGL(pa_merge_kernel, dim3((B * H + 3) / 4), dim3(256), 0, st, mg);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}
#endif  // LLM_TUNING
