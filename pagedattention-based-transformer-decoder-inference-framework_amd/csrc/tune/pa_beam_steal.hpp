// Beam-group attention with dynamic tile assignment (tuning build only:
// csrc/tune/pa_decode_tune.hip, LLM_BEAM_STEAL=1, plan form LLM_PA_FORM_STEAL).
// Measured slower than the shipped static BEAM form at every batch size
// (C4 launch 76.1-92.2 vs 65.3 us); kept for A/Bs.
//
// Same work as pa_split_kernel's BEAM form (one workgroup = the 4 beams of one
// sequence for one (head, split), wave i = beam i; a tile whose page id is the
// same in all 4 rows -- a forked prefix -- is fetched once per workgroup, each
// wave loading a quarter that the waves exchange through LDS; a beam-private
// tile is loaded by its own wave), with one change: which tiles a workgroup
// takes is decided while the launch runs.  The per-wave timeline of the BEAM
// form at C4 (scripts/beam_stamps.py) showed its static,
// cost-weighted split boundaries leaving a 37 -> 56 us tail in a 57 us launch
// (exit p10 36.8 us, p90 54.9 us) and 2.3-17 us before the first KV load (the
// 512-tile prefix scan behind beam_ids and page-table round trips).  Here:
//   * tiles go out in batches of KB, last tile first (the beam-private tail
//     is handed out first, the cheap shared tiles last): workgroup s starts on
//     items [s KB, (s + 1) KB) (no atomic before its first load), then takes the
//     next batch from a per-(sequence, head) counter (returning atomic add,
//     issued one batch ahead, published to the other waves through LDS at
//     mid-batch, so the next batch's page ids are in flight long before its
//     first tile is issued).  Workgroups that stream faster take more tiles.
//   * no prefix scan: a batch's page ids of the 4 rows (KB x 4 lanes, one
//     load) say per tile whether it is shared (all 4 equal) or private.
//   * every tile is one item for the whole workgroup: a shared tile is one
//     page (quarters through LDS, one barrier), a private tile is each wave's
//     own page of that tile; the next item's loads are in flight while the
//     current one is computed (two register stages, LDS double-buffered).
//   * the counters self-reset: every workgroup adds one arrival to done[gh]
//     after its last counter access, and the last arrival zeroes both, so
//     they are zero again for the next launch (the caller zeroes them once).
// Rows of a group whose contexts differ, or partial groups, run the static
// per-wave schedule of their own row (tiles [s pps, (s + 1) pps)).
// The arithmetic per tile is pa_split_kernel's (page_math below), so the
// partial states differ from the BEAM form's only in which tiles each split
// summed: the merged rows agree to fp32 rounding.
#pragma once

#include "pa_split.hpp"

namespace llm {

constexpr int kStealBatch = 4;  // tiles per batch (4 rows x KB ids: one load)

// MINW 4: 4 waves per SIMD (<= 128 VGPRs, D 128 / page 16), so the C4 grid
// (8 splits x 8 sequences x 16 heads = 1,024 workgroups of 4 waves) is one
// resident round; 16 KiB pages (D 256, or page 32) do not fit it and ask for 2.
// STAMPS (tuning build): per wave wid, stamps[wid * 8 + 0..7] = s_memrealtime
// at entry, before the first tile, after the last one, at exit; tiles
// computed, of them shared; 10 ns ticks spent at the mid-batch barriers; HW_ID.
template <int D, int TS, int KB = kStealBatch, int MINW = (TS * D <= 2048 ? 4 : 2),
          bool STAMPS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MINW))) void pa_beam_steal_kernel(
    PaSplitArgs a) {
  constexpr int EPL = 8;  // fp16
  constexpr int LPT = D / EPL;
  constexpr int TPI = 64 / LPT;
  constexpr int NI = TS / TPI;  // 1 KiB pieces per page and pool
  constexpr int PAGE_BYTES = TS * D * 2;
  constexpr int QP = NI / 2;  // pieces per wave of a shared tile (2 NI pieces over 4 waves)
  static_assert(KB >= 2 && 4 * KB <= 64, "steal form: batch size");
  static_assert(LPT >= 1 && LPT <= 64 && NI >= 2 && NI % 2 == 0, "steal form: D/TS");

  const unsigned long long t_entry = STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long t_first = 0, t_last = 0, t_mid = 0;
  int n_items = 0, n_shared = 0;
  const int lane = lane_id();
  const int gi = wave_id_uniform();  // beam within the group
  const int s = blockIdx.x % a.nsplit;
  const int gh = blockIdx.x / a.nsplit;
  const int h = gh % a.H;
  const int g0 = (gh / a.H) * 4;
  const int b = g0 + gi;
  const int c = lane % LPT;
  const int g = lane / LPT;

  // the group shares when all 4 rows exist, route to valid page-table rows and
  // hold equal contexts (uniform: every wave evaluates the same 4 rows)
  bool share = true;
  int prow[4];
  int Tg = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int bi = g0 + i;
    int ri = -1, Ti = 0;
    if (bi < a.B) {
      ri = a.beam_ids ? a.beam_ids[bi] : bi;
      Ti = a.context_lens ? a.context_lens[bi] : a.T;
      Ti = min(max(Ti, 0), a.T);
    }
    const bool rok = bi < a.B && ri >= 0 && ri < a.num_beams;
    prow[i] = rok ? (ri * a.H + h) * a.max_tiles : -1;
    if (!rok || (i > 0 && Ti != Tg)) share = false;
    if (i == 0) Tg = Ti;
  }
  if (b >= a.B) return;  // (no shared work: a partial group never shares)
  const size_t pidx = ((size_t)b * a.H + h) * a.nsplit + s;
  int Tb = a.context_lens ? a.context_lens[b] : a.T;
  Tb = min(max(Tb, 0), a.T);
  const int ntiles = min((Tb + TS - 1) / TS, a.max_tiles);

  float qv[EPL];
  {
    const float* qp = a.q + (size_t)b * a.q_stride + (size_t)h * D + c * EPL;
    const f32x4 q0 = *reinterpret_cast<const f32x4*>(qp);
    const f32x4 q1 = *reinterpret_cast<const f32x4*>(qp + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qv[e] = q0[e] * a.qscale;
      qv[4 + e] = q1[e] * a.qscale;
    }
  }
  float m = kNegSentinel, l = 0.f;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const uint32_t lane_off = (uint32_t)lane * 16u;

  // one page (pa_split_kernel's page_math): FULL = present and every token
  // inside the context
  auto page_math = [&](auto full_tag, const u32x4 (&kk)[NI], const u32x4 (&vv)[NI], bool ok,
                       int tok_base) {
    constexpr bool FULL = decltype(full_tag)::value;
    float sc[NI];
    bool valid[NI];
    float mloc = kNegSentinel;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) d = fmaf(qv[e], kv_at<LLM_F16>(kk[i], e), d);
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
      const u32x4 vraw = FULL || valid[i] ? vv[i] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] = fmaf(p, kv_at<LLM_F16>(vraw, e), acc[e]);
    }
    m = mnew;
  };
  auto tile_math = [&](const u32x4 (&kk)[NI], const u32x4 (&vv)[NI], int pg, int tile) {
    const bool ok = pg >= 0;
    const int tok_base = tile * TS + g;
    if (ok && (tile + 1) * TS <= Tb)
      page_math(std::true_type{}, kk, vv, ok, tok_base);
    else
      page_math(std::false_type{}, kk, vv, ok, tok_base);
  };
  auto rsrc = [&](const uint8_t* pool, int pg) {
    const bool ok = pg >= 0;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(pool + (size_t)(ok ? pg : 0) * a.page_stride), (short)0, ok ? PAGE_BYTES : 0,
        0x00020000);
  };
  auto valid_id = [&](int id) { return id >= a.num_pages ? -1 : id; };

  if (!share) {
    // the static per-wave schedule of this row (tiles [s pps, (s + 1) pps))
    const int r = prow[gi] >= 0 ? prow[gi] : -1;
    const int pps = row_pps(0, a.nsplit, ntiles);
    const int tile0 = s * pps;
    const int count = r >= 0 ? min(pps, ntiles - tile0) : 0;
    int pid0 = -1, pid1 = -1;
    if (lane < count) pid0 = valid_id(a.page_table[r + tile0 + lane]);
    if (64 + lane < count) pid1 = valid_id(a.page_table[r + tile0 + 64 + lane]);
    auto page_of = [&](int j) {
      return j < 64 ? __builtin_amdgcn_readlane(pid0, j) : __builtin_amdgcn_readlane(pid1, min(j - 64, 63));
    };
    auto issue = [&](u32x4 (&kk)[NI], u32x4 (&vv)[NI], int j) {
      const int pg = j < count ? page_of(min(j, kMaxPps - 1)) : -1;
      const auto krs = rsrc(a.k_pool, pg), vrs = rsrc(a.v_pool, pg);
#pragma unroll
      for (int i = 0; i < NI; ++i) kk[i] = __builtin_amdgcn_raw_buffer_load_b128(krs, lane_off + i * 1024, 0, kKvLoadAux);
#pragma unroll
      for (int i = 0; i < NI; ++i) vv[i] = __builtin_amdgcn_raw_buffer_load_b128(vrs, lane_off + i * 1024, 0, kKvLoadAux);
    };
    u32x4 kA[NI], vA[NI], kB[NI], vB[NI];
    if (count > 0) {
      issue(kA, vA, 0);
      for (int j = 0; j < count; j += 2) {
        issue(kB, vB, j + 1);
        tile_math(kA, vA, page_of(j), tile0 + j);
        if (j + 1 >= count) break;
        issue(kA, vA, j + 2);
        tile_math(kB, vB, page_of(min(j + 1, kMaxPps - 1)), tile0 + j + 1);
      }
    }
  } else {
    unsigned* ctr = a.steal + 2 * gh;  // [0] next dynamic batch (items past nsplit KB), [1] arrivals
    // items run last tile first: the beam-private tail (4 pages per tile) goes
    // out in the static batches and the dynamic ones end on shared tiles (one
    // page each), so the last batches taken are the cheapest
    auto tile_of = [&](int item) { return ntiles - 1 - item; };
    __shared__ __attribute__((aligned(16))) u32x4 kvbuf[2][2 * NI][64];
    __shared__ int next_lds[2];  // by batch parity: a slot is rewritten two batches later
    // lane j < 4 KB holds the page id of row j / KB, item t0 + j % KB
    auto load_ids = [&](int t0) {
      const int j = lane;
      const int it = t0 + j % KB;
      // raw: validated after the readlane (a compare here would wait for the load)
      return j < 4 * KB && it < ntiles ? a.page_table[prow[min(j / KB, 3)] + tile_of(it)] : -1;
    };
    // item k of a batch: shared (the page of all 4 rows) or private (this wave's own page)
    auto item_page = [&](int ids, int k, bool& shared) {
      const int p0 = valid_id(__builtin_amdgcn_readlane(ids, k));
      const int p1 = valid_id(__builtin_amdgcn_readlane(ids, KB + k));
      const int p2 = valid_id(__builtin_amdgcn_readlane(ids, 2 * KB + k));
      const int p3 = valid_id(__builtin_amdgcn_readlane(ids, 3 * KB + k));
      shared = p0 == p1 && p0 == p2 && p0 == p3;
      return shared ? p0 : gi == 0 ? p0 : gi == 1 ? p1 : gi == 2 ? p2 : p3;
    };
    struct Stage {
      u32x4 k[NI], v[NI];
    };
    // shared: this wave's quarter (pieces gi QP .. gi QP + QP - 1 of
    // [K pieces | V pieces]); private: the wave's whole page.  Every call
    // issues the same 2 NI load instructions (pieces not loaded get a
    // zero-record descriptor: no bytes move), so the compiler's wait for the
    // current item is a counted vmcnt(2 NI) behind the next item's loads,
    // never vmcnt(0); piece indices stay compile-time (no scratch).
    auto issue = [&](Stage& st, int pg, bool shared) {
      const auto krs = rsrc(a.k_pool, pg), vrs = rsrc(a.v_pool, pg);
      const auto none = rsrc(a.k_pool, -1);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        st.k[i] = __builtin_amdgcn_raw_buffer_load_b128(!shared || i / QP == gi ? krs : none,
                                                         lane_off + i * 1024, 0, kKvLoadAux);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        st.v[i] = __builtin_amdgcn_raw_buffer_load_b128(!shared || (NI + i) / QP == gi ? vrs : none,
                                                         lane_off + i * 1024, 0, kKvLoadAux);
    };
    int buf = 0;  // LDS buffer of the next shared item
    auto compute = [&](Stage& st, int pg, bool shared, int tile) {
      if (shared) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (i / QP == gi) kvbuf[buf][i][lane] = st.k[i];
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if ((NI + i) / QP == gi) kvbuf[buf][NI + i][lane] = st.v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          st.k[i] = kvbuf[buf][i][lane];
          st.v[i] = kvbuf[buf][NI + i][lane];
        }
        buf ^= 1;  // its next writer passes this item's barrier first
      }
      tile_math(st.k, st.v, pg, tile);
    };

    // Batch 0 is static (items [s KB, (s + 1) KB)); wave 0 asks for the next
    // batch when a batch starts and publishes the answer at mid-batch, where
    // the next batch's page ids start loading.  The body of one batch is
    // unrolled over its KB items, so stage indices and every wait are
    // compile-time (a counted vmcnt behind the next item's 2 NI loads).
    struct Item {
      bool have, shared;
      int pg, tile;
    };
    Stage st[2];
    int t0 = s * KB;
    int ids = load_ids(t0);
    unsigned got = 0;
    Item cur{t0 < ntiles, false, -1, tile_of(t0)};
    if (cur.have) cur.pg = item_page(ids, 0, cur.shared);
    issue(st[0], cur.have ? cur.pg : -1, cur.shared);
    int nb = 0;  // batches taken
    while (cur.have) {
      int nt0 = -1, nids = -1;
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        // the request for the next batch, and its answer at mid-batch, sit in
        // the same unrolled body: the wait for it is a counted vmcnt
        if (k == 0 && gi == 0 && lane == 0)
          got = __hip_atomic_fetch_add(ctr, (unsigned)KB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == KB / 2) {
          if (gi == 0 && lane == 0) next_lds[nb & 1] = (int)got;
          const unsigned long long tm0 = STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ull;
          __syncthreads();
          if constexpr (STAMPS) t_mid += __builtin_amdgcn_s_memrealtime() - tm0;
          nt0 = a.nsplit * KB + next_lds[nb & 1];
          nids = load_ids(nt0);
        }
        Item nx{false, false, -1, 0};
        if (k + 1 < KB) {
          if (t0 + k + 1 < ntiles) {
            nx.have = true;
            nx.tile = tile_of(t0 + k + 1);
            nx.pg = item_page(ids, k + 1, nx.shared);
          }
        } else if (nt0 < ntiles) {
          nx.have = true;
          nx.tile = tile_of(nt0);
          nx.pg = item_page(nids, 0, nx.shared);
        }
        issue(st[(k + 1) & 1], nx.have ? nx.pg : -1, nx.shared);
        if (cur.have) {
          if constexpr (STAMPS) {
            if (n_items == 0) t_first = __builtin_amdgcn_s_memrealtime();
            ++n_items;
            n_shared += cur.shared ? 1 : 0;
          }
          compute(st[k & 1], cur.pg, cur.shared, cur.tile);
        }
        cur = nx;
      }
      // on to the next batch (its first item is in flight in st[0])
      t0 = nt0;
      ids = nids;
      ++nb;
    }
    if constexpr (STAMPS) t_last = __builtin_amdgcn_s_memrealtime();
    // every wave is past its last counter access: one arrival per workgroup,
    // the last one resets both counters for the next launch
    __syncthreads();
    if (gi == 0 && lane == 0) {
      // the last batch request may be unused: retire it (vmcnt counts atomics
      // too) so the arrival below cannot overtake it past the reset
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old =
          __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (unsigned)a.nsplit - 1u) {
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  // merge the TPI row groups of the wave, write this split's partial of row b
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
  if (lane < LPT) {
    float* o = a.part_acc + pidx * D + c * EPL;
#pragma unroll
    for (int e = 0; e < EPL; e += 4) *reinterpret_cast<f32x4*>(o + e) = f32x4{acc[e], acc[e + 1], acc[e + 2], acc[e + 3]};
    if (lane == 0) {
      a.part_ml[pidx * 2] = m;
      a.part_ml[pidx * 2 + 1] = l;
    }
  }
  if constexpr (STAMPS) {
    if (lane == 0) {
      unsigned long long* o = a.stamps + ((size_t)blockIdx.x * 4 + gi) * 8;
      unsigned hw = 0, xcc = 0;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      o[0] = t_entry;
      o[1] = t_first;
      o[2] = t_last;
      o[3] = __builtin_amdgcn_s_memrealtime();
      o[4] = (unsigned long long)n_items;
      o[5] = (unsigned long long)n_shared;
      o[6] = t_mid;
      o[7] = ((unsigned long long)xcc << 32) | hw;
    }
  }
}

}  // namespace llm
