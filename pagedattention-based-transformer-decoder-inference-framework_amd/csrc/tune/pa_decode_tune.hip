// Tuning build only (make tune -> libllm_decoder_hip_tune.so; never in
// libllm_decoder_hip.so): the beam-group attention experiments that measured
// slower than the shipped BEAM form of pa_split_kernel, the
// tuning table pa_decode.hip reads (pa_tuning.hpp: the switches from the
// environment, and tune_launch_form, which routes a beam-group launch to the
// experiment switched on), and the pa_decode_tune A/B entry of the split
// kernel's register-stage / cache-policy variants (scripts/bench_kernels.py,
// scripts/tune_attention.py).
#include "tune/pa_decode_tune.hpp"
#include "tune/pa_beam_steal.hpp"
#include "pa_tuning.hpp"

namespace llm {

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

#ifndef BEAM4_MINW
#define BEAM4_MINW 2
#endif
#ifndef BEAM4_U
#define BEAM4_U 1
#endif

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


long long tune_beam4_resident_for(int D, int TS) {
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

hipError_t tune_launch_beam4(const PaSplitArgs& a, int D, int TS, hipStream_t st) {
  const int waves4 = ((a.B + 3) / 4) * a.H * a.nsplit;
  const dim3 grid((waves4 + 3) / 4), block(256);
  auto go = [&](auto d, auto ts) {
    constexpr int DD = decltype(d)::value, TT = decltype(ts)::value;
    if constexpr (TT * DD * 2 <= 8192)
      hipLaunchKernelGGL((pa_beam4_kernel<DD, TT, BEAM4_MINW, BEAM4_U>), grid, block, 0, st, a);
  };
  auto by_ts = [&](auto d) {
    if (TS == 16) go(d, std::integral_constant<int, 16>{});
    else go(d, std::integral_constant<int, 32>{});
  };
  switch (D) {
    case 32: by_ts(std::integral_constant<int, 32>{}); break;
    case 64: by_ts(std::integral_constant<int, 64>{}); break;
    case 128: by_ts(std::integral_constant<int, 128>{}); break;
    default: by_ts(std::integral_constant<int, 256>{}); break;
  }
  return hipGetLastError();
}

hipError_t tune_launch_beam_mfma(const PaSplitArgs& a, dim3 grid, hipStream_t st) {
  static const int dbg = env_int("LLM_BEAM_MFMA_DBG", 0);
  if (dbg == 1)
    hipLaunchKernelGGL(pa_beam_mfma_kernel<1>, grid, dim3(256), 0, st, a);
  else if (dbg == 2)
    hipLaunchKernelGGL(pa_beam_mfma_kernel<2>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(pa_beam_mfma_kernel<0>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t tune_launch_beam_loads_only(const PaSplitArgs& a, dim3 grid, hipStream_t st) {
#ifndef LLM_BEAM_CHUNK
#define LLM_BEAM_CHUNK 8192
#define LLM_BEAM_WAVES 0
#endif
  hipLaunchKernelGGL((pa_split_kernel<128, 16, false, LLM_BEAM_CHUNK, kKvLoadAux, 2, LLM_BEAM_WAVES,
                                      true, true>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

// The shipped BEAM form with its shared chunks delivered by an LDS-DMA ring
// of `ring` 8 KiB chunks (pa_split_kernel RING; LLM_BEAM_RING = 3 / 4 / 6 / 8,
// LLM_BEAM_DIAG = 2: the same with a trivial consumer).
hipError_t tune_launch_beam_ring(const PaSplitArgs& a, dim3 grid, hipStream_t st, int ring,
                                 bool load_only) {
  auto go = [&](auto r, auto lo) {
    constexpr int R = decltype(r)::value;
    constexpr bool LO = decltype(lo)::value;
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, LO, true, LLM_F16,
                                        true, false, false, R, false, true, true>),
                       grid, dim3(256), 0, st, a);
  };
  auto by_ring = [&](auto lo) {
    switch (ring) {
      case 3: go(std::integral_constant<int, 3>{}, lo); break;
      case 6: go(std::integral_constant<int, 6>{}, lo); break;
      case 8: go(std::integral_constant<int, 8>{}, lo); break;
      default: go(std::integral_constant<int, 4>{}, lo); break;
    }
  };
  if (load_only) by_ring(std::true_type{});
  else by_ring(std::false_type{});
  return hipGetLastError();
}

// The shipped BEAM form with per-wave timestamps (pa_split_kernel STAMPS,
// LLM_BEAM_STAMPS=1): entry / first KV load / shared prefix done / exit, and
// the wave's HW_ID, into a buffer pa_tune_stamps() copies out (diagnostics:
// allocates on first use, so not inside a graph capture).
static unsigned long long* g_stamps = nullptr;
static size_t g_stamps_cap = 0, g_stamps_waves = 0;

hipError_t tune_launch_beam_stamps(const PaSplitArgs& a0, dim3 grid, hipStream_t st) {
  const size_t waves = (size_t)grid.x * 4;
  if (waves > g_stamps_cap) {
    if (g_stamps) (void)hipFree(g_stamps);
    g_stamps = nullptr;
    g_stamps_cap = 0;
    if (hipMalloc(&g_stamps, waves * 5 * sizeof(unsigned long long)) != hipSuccess)
      return hipErrorOutOfMemory;
    g_stamps_cap = waves;
  }
  (void)hipMemsetAsync(g_stamps, 0, waves * 5 * sizeof(unsigned long long), st);
  PaSplitArgs a = a0;
  a.stamps = g_stamps;
  g_stamps_waves = waves;
  if (env_int("LLM_BEAM_INTERLEAVE", 1) == 0)
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, false, true, LLM_F16,
                                        true, false, false, 0, true>),
                       grid, dim3(256), 0, st, a);
  else if (env_int("LLM_BEAM_PRIO", 1) == 0)
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, false, true, LLM_F16,
                                        true, false, false, 0, true, true, false>),
                       grid, dim3(256), 0, st, a);

  else
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, false, true, LLM_F16,
                                        true, false, false, 0, true, true, true>),
                       grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

// The decoder's steal form (D 128, page 16) with per-wave stamps
// (pa_beam_steal_kernel STAMPS, 8 per wave; pa_tune_stamps8 copies them).
static unsigned long long* g_stamps8 = nullptr;
static size_t g_stamps8_cap = 0, g_stamps8_waves = 0;

hipError_t tune_launch_steal_stamps(const PaSplitArgs& a0, dim3 grid, hipStream_t st) {
  const size_t waves = (size_t)grid.x * 4;
  if (waves > g_stamps8_cap) {
    if (g_stamps8) (void)hipFree(g_stamps8);
    g_stamps8 = nullptr;
    g_stamps8_cap = 0;
    if (hipMalloc(&g_stamps8, waves * 8 * sizeof(unsigned long long)) != hipSuccess)
      return hipErrorOutOfMemory;
    g_stamps8_cap = waves;
  }
  (void)hipMemsetAsync(g_stamps8, 0, waves * 8 * sizeof(unsigned long long), st);
  PaSplitArgs a = a0;
  a.stamps = g_stamps8;
  g_stamps8_waves = waves;
  hipLaunchKernelGGL((pa_beam_steal_kernel<128, 16, kStealBatch, 4, true>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t tune_beam_mfma_occupancy(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, pa_beam_mfma_kernel<0>, 256, 0);
}

// ---------------------------------------------------------------------------
// The tuning table (pa_tuning.hpp): every switch read per launch (tests flip
// them in-process), except the beam balance, read once.
PaTuning pa_tuning() {
  static const int balance = [] {
    const int x = env_int("LLM_BEAM_BALANCE16", 44);
    return x >= 16 ? x : 0;
  }();
  static const int mfma_balance = [] {
    const int x = env_int("LLM_BEAM_MFMA_BALANCE16", 64);
    return x >= 16 ? x : 0;
  }();
  PaTuning t;
  t.wg_merge = env_int("LLM_WG_MERGE", 1) != 0;
  t.oproj_fuse = env_int("LLM_OPROJ_FUSE", 1) != 0;
  t.beam4 = env_int("LLM_BEAM4", 0) != 0;
  t.beam_mfma = env_int("LLM_BEAM_MFMA", 0) != 0;
  t.beam_steal = env_int("LLM_BEAM_STEAL", 0) == 1;
  t.beam_balance16 = balance;
  t.beam_mfma_balance16 = mfma_balance;
  t.beam_nsplit = env_int("LLM_BEAM_NSPLIT", 0);
  t.wgm_splits = env_int("LLM_WGM_SPLITS", 0);
  t.beam4_splits = env_int("LLM_BEAM4_SPLITS", 0);
  t.beam_smaj = env_int("LLM_BEAM_SMAJ", 1) != 0;
  return t;
}

bool tune_beam_occupancy(int D, int TS, int* blocks, hipError_t* e) {
  if (D != 128 || TS != 16 || !pa_tuning().beam_mfma) return false;
  *e = tune_beam_mfma_occupancy(blocks);
  return true;
}

unsigned* tune_steal_counters(size_t n) {
  static unsigned* buf = nullptr;
  static size_t cap = 0;
  if (!pa_tuning().beam_steal) return nullptr;
  if (n > cap) {
    if (buf) (void)hipFree(buf);
    buf = nullptr;
    cap = 0;
    if (hipMalloc(&buf, n * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(buf, 0, n * sizeof(unsigned)) != hipSuccess) return nullptr;
    cap = n;
  }
  return buf;
}

namespace {
// the steal form (pa_beam_steal_kernel) of one (D, TS): LLM_STEAL_KB tiles per
// batch, LLM_STEAL_MINW=3 lifts the 128-VGPR cap, LLM_BEAM_STAMPS=1 stamps
template <int D, int TS>
hipError_t launch_steal(const PaSplitArgs& a, dim3 grid, hipStream_t st) {
  if constexpr (D == 128 && TS == 16) {
    if (env_int("LLM_BEAM_STAMPS", 0) == 1) return tune_launch_steal_stamps(a, grid, st);
  }
  const int kb = env_int("LLM_STEAL_KB", kStealBatch);
  if (env_int("LLM_STEAL_MINW", 0) == 3)
    hipLaunchKernelGGL((pa_beam_steal_kernel<D, TS, kStealBatch, 3>), grid, dim3(256), 0, st, a);
  else if (kb == 2) hipLaunchKernelGGL((pa_beam_steal_kernel<D, TS, 2>), grid, dim3(256), 0, st, a);
  else if (kb == 8) hipLaunchKernelGGL((pa_beam_steal_kernel<D, TS, 8>), grid, dim3(256), 0, st, a);
  else if (kb == 16) hipLaunchKernelGGL((pa_beam_steal_kernel<D, TS, 16>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((pa_beam_steal_kernel<D, TS>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}
}  // namespace

bool tune_launch_form(const PaSplitArgs& a, int D, int TS, dim3 grid, hipStream_t st,
                      hipError_t* e) {
  if (a.beam4) {  // pa_beam4_kernel: one wave per (group, head, split)
    *e = tune_launch_beam4(a, D, TS, st);
    return true;
  }
  if (a.steal && steal_shape_ok(D, TS)) {  // dynamic tile assignment (pa_beam_steal.hpp)
    if (D == 64 && TS == 16) *e = launch_steal<64, 16>(a, grid, st);
    else if (D == 128 && TS == 16) *e = launch_steal<128, 16>(a, grid, st);
    else if (D == 32 && TS == 32) *e = launch_steal<32, 32>(a, grid, st);
    else if (D == 64 && TS == 32) *e = launch_steal<64, 32>(a, grid, st);
    else if (D == 128 && TS == 32) *e = launch_steal<128, 32>(a, grid, st);
    else return false;
    return true;
  }
  if (D != 128 || TS != 16) return false;
  const PaTuning t = pa_tuning();
  if (t.beam_mfma) {
    PaSplitArgs am = a;
    am.balance16 = t.beam_mfma_balance16;
    *e = tune_launch_beam_mfma(am, grid, st);
    return true;
  }
  if (env_int("LLM_BEAM_DIAG", 0) == 1) {  // this form's loads, staging and barriers only
    *e = tune_launch_beam_loads_only(a, grid, st);
    return true;
  }
  if (env_int("LLM_BEAM_STAMPS", 0) == 1) {  // per-wave timestamps (scripts/beam_stamps.py)
    *e = tune_launch_beam_stamps(a, grid, st);
    return true;
  }
  const int ring = env_int("LLM_BEAM_RING", 0);
  if (ring > 0) {  // shared chunks through an LDS-DMA ring
    *e = tune_launch_beam_ring(a, grid, st, ring, env_int("LLM_BEAM_DIAG", 0) == 2);
    return true;
  }
  if (env_int("LLM_BEAM_PRIO", 1) == 0) {  // interleaved splits without the priority ranking
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, false, true, LLM_F16,
                                        true, false, false, 0, false, true, false>),
                       grid, dim3(256), 0, st, a);
    *e = hipGetLastError();
    return true;
  }
  if (env_int("LLM_BEAM_INTERLEAVE", 1) == 0) {  // round 4's contiguous cost-balanced splits
    hipLaunchKernelGGL((pa_split_kernel<128, 16, false, 8192, kKvLoadAux, 2, 0, false, true>),
                       grid, dim3(256), 0, st, a);
    *e = hipGetLastError();
    return true;
  }
  return false;
}

}  // namespace llm

using namespace llm;

// Tuning hook: the last steal-form stamps (8 per wave) into host; returns the
// waves copied (-1: none recorded).
extern "C" long long pa_tune_stamps8(unsigned long long* host, long long max_waves) {
  if (!g_stamps8 || !host) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const size_t n = std::min<size_t>((size_t)max_waves, g_stamps8_waves);
  if (hipMemcpy(host, g_stamps8, n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return -1;
  return (long long)n;
}

// Tuning hook: the last LLM_BEAM_STAMPS launch's per-wave stamps (5 per wave,
// pa_split_kernel STAMPS) into host (room for max_waves); returns the waves
// copied (-1: none recorded).
extern "C" long long pa_tune_stamps(unsigned long long* host, long long max_waves) {
  if (!g_stamps || !host) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const size_t n = std::min<size_t>((size_t)max_waves, g_stamps_waves);
  if (hipMemcpy(host, g_stamps, n * 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return -1;
  return (long long)n;
}

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
  return pa_merge_splits_internal(a.part_acc, a.part_ml, out, context_lens, B, H, D, T, 16, pps,
                                  nsplit, kv->max_tiles, st);
}
