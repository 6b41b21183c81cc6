// Paged decode attention: the split kernel (device code of pa_decode.hip,
// shared with the tuning build's csrc/tune/pa_decode_tune.hip).
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
#pragma once

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
  // beam-group launches with dynamic tile assignment (tuning build, tune/pa_beam_steal.hpp):
  // per (sequence group, head) the next-batch counter and the arrival count,
  // zero at launch, left at zero by the launch
  unsigned* steal;
  // tuning (pa_split_kernel STAMPS): per wave wid, s_memrealtime (100 MHz) at
  // entry, at the first KV load, after the shared-prefix chunks, at exit, and
  // the wave's HW_ID (CU / SIMD / XCC placement): stamps[wid * 5 + 0..4]
  unsigned long long* stamps;
  // BEAM: split-major workgroup order (blockIdx = s * groups * H + group * H +
  // head) instead of ((group * H + head) * nsplit + s).  A CU's 4 resident
  // workgroups (blockIdx b, b + 256, b + 512, b + 768 at C4) are then 4 split
  // pairs of 4 (group, head)s rather than 4 sequence pairs, and the splits of
  // one (group, head) share an XCD (blockIdx mod 8) and its L2.
  int smaj;  // (last: the earlier fields keep their kernel-argument offsets)
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
// INTERLEAVE (BEAM, dynamic splits): split s holds the row's tiles s, s + NS,
// s + 2 NS, ... instead of a contiguous range.  Every split then holds the
// same mix of shared-prefix and beam-private tiles (C4: 30 shared + 2 private
// of 257), so the splits finish together without a cost model, and the split's
// page ids are requested at entry (their tile indices need no context length)
// instead of after a 512-tile prefix scan and its barrier.
// PRIO (BEAM): wave priority falls with the shared-chunk progress (3 at entry,
// 2 / 1 / 0 after a quarter / half / three quarters).  A CU holds 4 beam
// workgroups dispatched one after another; at equal priority the SIMD arbiter
// favours the oldest waves, so the first workgroup placed on a CU finishes
// long before the last (C4 stamps: exits 34 / 39 / 45 / 52 us by dispatch
// slot), and the last runs alone with 16 KiB in flight.  Priority outranks age
// (MI355X_MICROARCH.md, two waves per SIMD, item 4): the laggards catch up.
template <int D, int TS, bool DIRECT, int CHUNK_BYTES = 16384, int AUX = kKvLoadAux,
          int STAGES = 2, int MIN_WAVES = 0, bool LOAD_ONLY = false, bool BEAM = false,
          int KVT = LLM_F16, bool FULLPATH = true, bool WGM = false, bool OPROJ = false,
          int RING = 0, bool STAMPS = false, bool INTERLEAVE = false, bool PRIO = false>
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
  static_assert(!INTERLEAVE || BEAM, "interleaved splits are a beam-group form");
  constexpr bool IL = BEAM && INTERLEAVE;
  static_assert(!OPROJ || (WGM && KVT == LLM_F16), "the fused o_proj is a workgroup-merge form");
  const unsigned long long t_entry = STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ull;
  if constexpr (BEAM && PRIO) __builtin_amdgcn_s_setprio(3);
  const int lane = lane_id();
  const int wid = blockIdx.x * (WGM ? a.nsplit : 4) + wave_id_uniform();
  const int G = BEAM ? 4 : WGM ? 1 : a.group;
  const int gi = wid % G;  // row within the group (fastest: adjacent waves)
  const int rest = wid / G;
  const int GH = BEAM && a.smaj ? ((a.B + 3) / 4) * a.H : 1;
  const int s = BEAM && a.smaj ? rest / GH : rest % a.nsplit;
  const int gh = BEAM && a.smaj ? rest % GH : rest / a.nsplit;
  const int h = gh % a.H;
  const int b = (gh / a.H) * G + gi;
  // BEAM: the shared path runs only when all 4 rows exist, route to a valid
  // page-table row and hold the same context (a uniform decision: every wave
  // of the workgroup evaluates the same 4 rows, before any early return).
  // The 4 rows' beam ids and contexts are loaded side by side (no early exit:
  // a row-by-row loop made them 4 dependent round trips), and this wave's own
  // row's first kPfx page-table ids (the prefix scan below) are requested as
  // soon as its beam id is known, before the contexts decide whether the
  // group shares: under the other workgroups' KV streams each dependent round
  // trip here cost about a microsecond of start-up.
  constexpr int kPfx = 512;
  bool share = false;
  int grow[4] = {0, 0, 0, 0};  // BEAM: the group's page-table rows
  int idv[BEAM && !IL ? kPfx / 64 : 1];
  const bool pfx_on = BEAM && !IL && a.balance16 >= 16 && a.pps == 0 && a.nsplit > 1;
  // IL: interleaved splits (dynamic split length, groups that share: 4 rows
  // of equal context; ragged groups keep the plain schedule's contiguous
  // splits); ilp0 / ilp1 = this wave's row's page ids of tiles s + NS lane and
  // s + NS (64 + lane), requested before `share` is known
  bool il = IL && a.pps == 0 && a.nsplit > 1;
  int ilp0 = -1, ilp1 = -1;
  if constexpr (BEAM) {
    const int g0 = b - gi;
    int Ti[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int bi = min(g0 + i, a.B - 1);
      grow[i] = a.beam_ids ? a.beam_ids[bi] : bi;
      Ti[i] = a.context_lens ? a.context_lens[bi] : a.T;
    }
    const bool own_ok = grow[gi] >= 0 && grow[gi] < a.num_beams;
    const int32_t* prow = a.page_table + ((size_t)(own_ok ? grow[gi] : 0) * a.H + h) * a.max_tiles;
    if constexpr (IL) {
      const int t0 = s + a.nsplit * lane, t1 = s + a.nsplit * (64 + lane);
      ilp0 = il && own_ok && t0 < a.max_tiles ? prow[t0] : -1;
      ilp1 = il && own_ok && t1 < a.max_tiles ? prow[t1] : -1;
    } else {
      const int lim0 = min(a.max_tiles, kPfx);
#pragma unroll
      for (int k = 0; k < kPfx / 64; ++k) {
        const int t = 64 * k + lane;
        idv[k] = pfx_on && own_ok && t < lim0 ? prow[t] : -1;
      }
    }
    share = g0 + 3 < a.B;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      share = share && grow[i] >= 0 && grow[i] < a.num_beams &&
              min(max(Ti[i], 0), a.T) == min(max(Ti[0], 0), a.T);
    il = il && share;
  }
  if (b >= a.B) return;
  const int bh = b * a.H + h;
  const size_t pidx = (size_t)bh * a.nsplit + s;  // partial-state slot
  const int r = a.beam_ids ? a.beam_ids[b] : b;
  int Tb = a.context_lens ? a.context_lens[b] : a.T;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + TS - 1) / TS, a.max_tiles);
  int tile0, count;
  // tiles of the split: tile0 + j * tstride, j < count
  int tstride = 1;
  if (IL && il) {
    tile0 = s;
    tstride = a.nsplit;
    count = ntiles > s ? (ntiles - s + a.nsplit - 1) / a.nsplit : 0;
  } else {
    const int pps = row_pps(a.pps, a.nsplit, ntiles);
    tile0 = s * pps;
    count = min(pps, ntiles - tile0);
  }
  // BEAM: the page ids of the group's 4 rows, tiles [0, pfx_lim), read once
  // by the prefix scan below and reused for this split's page ids
  __shared__ int pfx_lds[BEAM && !IL ? 4 : 1][BEAM && !IL ? kPfx : 1];
  int pfx_lim = 0;
  if constexpr (BEAM && !IL) {
    // Cost-balanced splits: a split's beam-private tiles are loaded by every
    // wave (4x the per-wave bytes of a shared tile, which the workgroup loads
    // once), so equal tile counts leave the splits holding the private tail
    // slowest.  The group's shared prefix (leading tiles whose page ids agree
    // in all 4 rows) is found cooperatively and the boundaries put equal cost
    // (shared 16, private balance16) in each split.  Every input is uniform
    // over the workgroup, so all splits of a row (one workgroup each) derive
    // the same partition.  The first kPfx tiles' ids of every row are loaded
    // in ONE round trip (8 loads per lane in flight, then one barrier): the
    // 64-tile rounds this replaced cost a dependent page-table load and two
    // barriers each before the first KV load could issue.
    if (share && pfx_on && ntiles > 0) {
      const int32_t* prow = a.page_table + ((size_t)grow[gi] * a.H + h) * a.max_tiles;
      const int lim = min(ntiles, kPfx);
#pragma unroll
      for (int k = 0; k < kPfx / 64; ++k) {
        const int t = 64 * k + lane;
        pfx_lds[gi][t] = t >= lim || idv[k] >= a.num_pages ? -1 : idv[k];
      }
      __syncthreads();
      int nsh_t = 0;
      for (int blk = 0; blk < lim; blk += 64) {
        const int t = blk + lane;
        const bool eq = t < lim && pfx_lds[0][t] == pfx_lds[1][t] && pfx_lds[0][t] == pfx_lds[2][t] &&
                        pfx_lds[0][t] == pfx_lds[3][t];
        const uint64_t mk = __ballot(eq);
        const int run = mk == ~0ull ? 64 : __builtin_ctzll(~mk);
        nsh_t = blk + run;
        if (run < 64) break;
      }
      nsh_t = min(nsh_t, lim);
      pfx_lim = lim;
      // a shared run past the first kPfx tiles: continue 64 tiles per round
      if (nsh_t == lim && lim < ntiles) for (int blk = kPfx;; blk += 64) {
        __shared__ int pfx2_lds[4][64];
        const int t = blk + lane;
        int id = -1;
        if (t < ntiles) {
          id = prow[t];
          if (id >= a.num_pages) id = -1;
        }
        pfx2_lds[gi][lane] = id;
        __syncthreads();
        const bool eq = t < ntiles && pfx2_lds[0][lane] == pfx2_lds[1][lane] &&
                        pfx2_lds[0][lane] == pfx2_lds[2][lane] && pfx2_lds[0][lane] == pfx2_lds[3][lane];
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
  if (IL && il) {  // requested at entry (r is the group's row gi)
    pid0 = lane < count && ilp0 < a.num_pages ? ilp0 : -1;
    pid1 = 64 + lane < count && ilp1 < a.num_pages ? ilp1 : -1;
  } else if (BEAM && tile0 + count <= pfx_lim) {  // (r is the group's row gi: read by the prefix scan)
    if (lane < count) pid0 = pfx_lds[gi][tile0 + lane];
    if (64 + lane < count) pid1 = pfx_lds[gi][tile0 + 64 + lane];
  } else if (r >= 0 && r < a.num_beams) {
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
      const int tile = tile0 + j * (IL ? tstride : 1);
      const int tok_base = tile * TS + g;
      if (FULLPATH && ok && (tile + 1) * TS <= Tb)
        page_math(std::true_type{}, u, ok, tok_base);
      else
        page_math(std::false_type{}, u, ok, tok_base);
    }
  };

  const int nchunks = (count + U - 1) / U;
  int ch0 = 0;  // first chunk of the per-wave direct path
  unsigned long long t_load = 0, t_shared = 0;
  if constexpr (STAMPS) {
    (void)page_of(0);  // the page ids have arrived
    t_load = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (BEAM) {
    static_assert(NR % 2 == 0, "beam prefetch splits a chunk's 2*NR pieces in quarters");
    constexpr int QP = NR / 2;  // pieces per wave per chunk
    static_assert(RING == 0 || (RING >= 3 && (RING - 2) * QP < 64), "ring of 3+ chunks");
    __shared__ int pid_lds[4][128];
    __shared__ __attribute__((aligned(16))) u32x4 kvbuf[RING > 0 ? RING : 2][2 * NR][64];
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
      if constexpr (RING > 0) {
        // LDS-DMA ring (tuning): each wave's quarter of chunk cc goes straight
        // from HBM into ring slot cc % RING (buffer_load ... lds: lane-linear,
        // no VGPR stage, no ds_write pass), RING - 1 chunks in flight per
        // workgroup.  Per chunk: the wave's own pieces of cc are retired by a
        // counted vmcnt (the later chunks stay in flight), one raw barrier
        // publishes every wave's pieces and retires the reads of slot
        // (cc - 1) % RING, which the next DMA then refills.  Chunks past the
        // shared prefix are issued with zero records (no bytes, no fault) so
        // every wait counts the same number of loads.
        if (nsh > 0) {
          auto dma = [&](int cc) {
            const int slot = cc % RING;
#pragma unroll
            for (int t = 0; t < QP; ++t) {
              const int q = gi * QP + t;
              const int pi = q % NR;
              const int u = pi / NI, i = pi % NI;
              const int j = cc * U + u;
              const int pg = page_of(min(j, kMaxPps - 1));
              const bool ok = cc < nsh && j < count && pg >= 0;
              const size_t off = (size_t)(ok ? pg : 0) * a.page_stride;
              const uint8_t* pool = q < NR ? a.k_pool : a.v_pool;
              const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(pool + off), (short)0,
                                                                ok ? PAGE_BYTES : 0, 0x00020000);
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  rs, (__attribute__((address_space(3))) void*)&kvbuf[slot][q][0], 16,
                  lane_off + i * 1024, 0, 0, AUX);
            }
          };
#pragma unroll
          for (int c0 = 0; c0 < RING - 1; ++c0) dma(c0);
          for (int cc = 0; cc < nsh; ++cc) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((RING - 2) * QP)
                         : "memory");
            const int cur = cc % RING;
            u32x4 kk[NR], vv[NR];
            // the slot's reads as one asm block (+ lgkmcnt(0)): read through
            // plain LDS loads, the compiler would retire every DMA in flight
            // (vmcnt(0)) before them, which is the ring's whole point lost
            const uint32_t ra = (uint32_t)(size_t)(
                __attribute__((address_space(3))) void*)&kvbuf[cur][0][lane];
            static_assert(NR == 4, "the ring's asm reads are written for 8 KiB chunks");
            asm volatile(
                "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:1024\n\t"
                "ds_read_b128 %2, %8 offset:2048\n\tds_read_b128 %3, %8 offset:3072\n\t"
                "ds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %8 offset:5120\n\t"
                "ds_read_b128 %6, %8 offset:6144\n\tds_read_b128 %7, %8 offset:7168\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(kk[0]), "=&v"(kk[1]), "=&v"(kk[2]), "=&v"(kk[3]), "=&v"(vv[0]), "=&v"(vv[1]),
                  "=&v"(vv[2]), "=&v"(vv[3])
                : "v"(ra)
                : "memory");
            dma(cc + RING - 1);
            compute(kk, vv, cc * U);
          }
          // the zero-record tail loads write LDS the ring no longer reads;
          // retire them before the direct path's own loads are counted
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if (nsh > 0) {
        u32x4 qr[QP];
        quarter(qr, 0);
#pragma unroll
        for (int t = 0; t < QP; ++t) kvbuf[0][gi * QP + t][lane] = qr[t];
        if (nsh > 1) quarter(qr, 1);
        __syncthreads();
        for (int cc = 0; cc < nsh; ++cc) {
          if constexpr (PRIO) {  // (uniform: nsh and cc are)
            if (cc == nsh / 4) __builtin_amdgcn_s_setprio(2);
            if (cc == nsh / 2) __builtin_amdgcn_s_setprio(1);
            if (cc == (3 * nsh) / 4) __builtin_amdgcn_s_setprio(0);
          }
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
    // the priority raised at entry falls with the shared-chunk progress; a
    // workgroup that shares nothing (ragged group, nsh == 0) or whose last
    // quarter of chunks set nothing drops it here, so it never streams its
    // private tiles at top priority past the shared-prefix laggards
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (STAMPS) t_shared = __builtin_amdgcn_s_memrealtime();
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
  if constexpr (STAMPS) {
    if (lane == 0) {
      unsigned long long* st = a.stamps + (size_t)wid * 5;
      st[0] = t_entry;
      st[1] = t_load;
      st[2] = t_shared;
      st[3] = __builtin_amdgcn_s_memrealtime();
      unsigned hw = 0, xcc = 0;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      st[4] = ((unsigned long long)xcc << 32) | hw;
    }
  }
}

}  // namespace llm
