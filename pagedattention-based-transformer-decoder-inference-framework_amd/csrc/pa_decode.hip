// Paged decode attention for gfx950 (CDNA4): launch planning (split counts,
// forms), the split merges and the C entry points (pa_decode,
// pa_decode_grouped, pa_decode_plan).  The split kernel itself, and the design
// notes of the scan, are in pa_split.hpp; the tuning build's experiment
// kernels and A/B entry are in csrc/tune/pa_decode_tune.hip.
#include "pa_split.hpp"
#include "pa_tuning.hpp"

namespace llm {

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

// One head's split merge (flash-decoding LSE combine) by one wave, DPL =
// output dims per lane (D / 64, at least 1).  The head's split weights (m, l),
// lane-parallel (lane holds splits lane and 64 + lane), and the partials of
// its first BATCH splits are loaded together: every address depends on the
// launch's arguments only (clamped to its nsplit), so they issue with the
// caller's context_lens load and a merge costs one memory round trip (splits
// beyond the batch: one more per 8).  The row's split count ns masks the
// values afterwards (splits past ns may hold stale bits).  Summation order
// s = 0, 1, ... (sequential) for L and for every output; split s's (l, w) come
// from lane s by readlane.  acc[j] * the returned 1 / L is the output at dim
// lane + 64 j; a head with no partial returns acc = 0.
template <int DPL, int BATCH>
__device__ __forceinline__ float merge_head(const float* ml, const float* pa, int nsplit, int ns,
                                            int D, float (&acc)[DPL]) {
  const int lane = lane_id();
  const int nsl = max(nsplit - 1, 0);
  const float m0r = ml[2 * min(lane, nsl)], l0r = ml[2 * min(lane, nsl) + 1];
  const float m1r = ml[2 * min(64 + lane, nsl)], l1r = ml[2 * min(64 + lane, nsl) + 1];
  float v[BATCH][DPL];
#pragma unroll
  for (int s2 = 0; s2 < BATCH; ++s2)
#pragma unroll
    for (int j = 0; j < DPL; ++j)
      v[s2][j] = pa[(size_t)min(s2, nsl) * D + min(lane + 64 * j, D - 1)];
  const float m0 = lane < ns ? m0r : kNegSentinel;
  const float m1 = 64 + lane < ns ? m1r : kNegSentinel;
  const float l0 = lane < ns ? l0r : 0.f;
  const float l1 = 64 + lane < ns ? l1r : 0.f;
#pragma unroll
  for (int s2 = 0; s2 < BATCH; ++s2)
#pragma unroll
    for (int j = 0; j < DPL; ++j) v[s2][j] = s2 < ns ? v[s2][j] : 0.f;
#pragma unroll
  for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
  const float M = ln_wave_max(fmaxf(m0, m1));
  if (ns <= 0 || M <= 0.5f * kNegSentinel) return 0.f;
  const float w0 = lane < ns ? __builtin_amdgcn_exp2f(m0 - M) : 0.f;
  const float w1 = 64 + lane < ns ? __builtin_amdgcn_exp2f(m1 - M) : 0.f;
  float L = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < BATCH; ++s2)
    if (s2 < ns) {
      const float ls = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l0), s2));
      const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));
      L += ls * ws;
    }
  for (int s2 = BATCH; s2 < ns; ++s2) {
    const float ls = s2 < 64 ? __shfl(l0, s2, 64) : __shfl(l1, s2 - 64, 64);
    const float ws = s2 < 64 ? __shfl(w0, s2, 64) : __shfl(w1, s2 - 64, 64);
    L += ls * ws;
  }
#pragma unroll
  for (int s2 = 0; s2 < BATCH; ++s2) {
    const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w0), s2));  // 0 past ns
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] += v[s2][j] * ws;
  }
  for (int s0 = BATCH; s0 < ns; s0 += 8) {  // long split lists
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
      const int d = lane + 64 * j;
      float u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = (s0 + k < ns && d < D) ? pa[(size_t)(s0 + k) * D + d] : 0.f;
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
  return 1.0f / (L + 1e-6f);
}

// Split merge, fp32 output: one wave per (b, h), 4 per workgroup.  The first
// 16 splits' partials come in the first round trip (the 8-row C3 step merges
// 16 splits per head: 8.0 us per launch when the (m, l) and partial loads
// were issued split by split).
struct PaMergeArgs {
  const float* part_acc;
  const float* part_ml;
  float* out;
  const int32_t* context_lens;
  int B, H, D, T, TS, pps, nsplit, max_tiles;
};

template <int DPL>
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
  float acc[DPL];
  const float inv = merge_head<DPL, 16>(a.part_ml + (size_t)bh * a.nsplit * 2,
                                        a.part_acc + (size_t)bh * a.nsplit * a.D, a.nsplit, ns,
                                        a.D, acc);
  float* o = a.out + (size_t)bh * a.D;
#pragma unroll
  for (int j = 0; j < DPL; ++j) {
    const int d = lane + 64 * j;
    if (d < a.D) o[d] = acc[j] * inv;
  }
}

// Splits per first round trip of pa_merge_row_kernel's heads.
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
    float acc[DPL];
    const float inv = merge_head<DPL, kMergeBatch>(a.part_ml + bh * a.nsplit * 2,
                                                   a.part_acc + bh * a.nsplit * a.D, a.nsplit, ns,
                                                   a.D, acc);
    float* dst = row + h * a.D;
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

}  // namespace

// The FP16 decoder's o_proj fused into the workgroup merge (decoder.cpp
// oproj_fusable); LLM_OPROJ_FUSE=0 (tuning build) restores the o_proj GEMM.
bool oproj_fuse_on() { return pa_tuning().oproj_fuse; }
bool beam_steal_on() { return pa_tuning().beam_steal; }

namespace {

// The experiment forms of beam-group launches (pa_beam4_kernel,
// pa_beam_mfma_kernel, the steal form, ...) exist only in the tuning build
// (csrc/tune/pa_decode_tune.hip, switched by pa_tuning.hpp).  All measured
// slower than the LDS-staged BEAM form of pa_split_kernel (C4 launch with
// merge: beam4 69.2 us at 16 splits, 74.2 with two pages per register stage,
// 82.3 at 12 splits, against 67.6 us; MFMA 69.8 vs 60.8 us; steal 76-92 vs
// 65.3 us).

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
  if (a.group == 4 && !direct && ST == 2) {
    // 8 KiB register stages: 112 VGPRs, 4 waves per SIMD.  The 16 KiB form
    // (179 VGPRs, 2 waves) spent 27 % of its wave time in issue stalls and
    // 20 % parked (SQ PMC, scripts/gpu_sq_pmc.sh); same-box A/B of the C4
    // launch: 72-74 vs 76 us (scripts/ab_attention_lib.py, -DLLM_BEAM_CHUNK=)
#ifndef LLM_BEAM_CHUNK
#define LLM_BEAM_CHUNK 8192
#define LLM_BEAM_WAVES 0
#endif
    hipError_t te;
    if (tune_launch_form(a, D, TS, grid, st, &te)) {  // tuning build: an experiment form
      *beam = true;
      return te;
    }
    hipLaunchKernelGGL((pa_split_kernel<D, TS, false, LLM_BEAM_CHUNK, kKvLoadAux, 2, LLM_BEAM_WAVES,
                                        false, true, LLM_F16, true, false, false, 0, false, true, true>),
                       grid, block, 0, st, a);
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
  const dim3 grid((B * H + 3) / 4);
  if (D <= 64)
    hipLaunchKernelGGL(pa_merge_kernel<1>, grid, dim3(256), 0, st, mg);
  else if (D <= 128)
    hipLaunchKernelGGL(pa_merge_kernel<2>, grid, dim3(256), 0, st, mg);
  else
    hipLaunchKernelGGL(pa_merge_kernel<4>, grid, dim3(256), 0, st, mg);
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
template <int D, int TS>
hipError_t beam_occupancy(int* blocks) {
  hipError_t e;
  if (tune_beam_occupancy(D, TS, blocks, &e)) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(
      blocks, pa_split_kernel<D, TS, false, LLM_BEAM_CHUNK, kKvLoadAux, 2, LLM_BEAM_WAVES, false, true,
                              LLM_F16, true, false, false, 0, false, true, true>,
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
  const PaTuning tn = pa_tuning();
  int nsplit = choose_nsplit(B, H, ntiles_max, pps_fixed, resident_launch);
  // fp32 rows whose launch is exactly one resident round of more splits than
  // a workgroup merge holds (C3's model at 8 rows per GPU: 128 (row, head)
  // pairs x 16 splits of 33 pages = 2,048 waves): half the splits, twice as
  // long, still split + merge.  Standalone (scripts/tune_attention.py --B 8,
  // profiles/r05/attention_b8_split_sweep.txt): 85.6 -> 84.3 us, the
  // loads-only form 83.7 / 83.4 us at either count.
  const bool half_round = f32_rows && row_group == 1 && pps_fixed <= 0 &&
                          kv->kv_dtype == LLM_F16 && nsplit > kWgmMaxSplits &&
                          (long long)B * H * nsplit == resident_launch &&
                          (ntiles_max + nsplit - 1) / nsplit <= 2 * kShortPps;
  if (half_round) nsplit = (nsplit + 1) / 2;
  const bool wgm_ok = ((row_out && rows->out16 && !rows->q) || oproj || f32_rows) && row_group == 1 &&
                      kv->kv_dtype == LLM_F16 && tn.wg_merge && !half_round;
  if (wgm_ok && pps_fixed <= 0 && !f32_rows) {
    const int nw = choose_nsplit(B, H, ntiles_max, 0, resident_launch, kWgmShortPps);
    if (nw >= 2 && nw <= kWgmMaxSplits) nsplit = nw;
  }
  if (wgm_ok && pps_fixed <= 0 && f32_rows && nsplit >= 2) {
    int nw = 2;
    while (nw < nsplit && nw < kWgmMaxSplits) nw *= 2;
    if (nw >= nsplit && (long long)nw * kMaxPps >= ntiles_max) nsplit = nw;
  }
  // tuning build: forced split counts of beam-group launches and of the
  // workgroup-merge eligible ones (fp16 row outputs, dynamic splits)
  if (row_group == 4 && pps_fixed <= 0) {
    const int f = tn.beam_nsplit;
    if (f >= 2 && (long long)f * kMaxPps >= ntiles_max) nsplit = std::min(f, kMaxSplits);
  }
  if (rows && (rows->out16 || oproj || f32_rows) && !rows->q && row_group == 1 && pps_fixed <= 0) {
    const int f = tn.wgm_splits;
    if (f >= 2 && f <= kWgmMaxSplits && (long long)f * kMaxPps >= ntiles_max) nsplit = f;
  }
  // beam groups of 4 rows (fp16 pages <= 8 KiB, dynamic splits): pa_beam4_kernel,
  // one wave per (group, head, split), splits sized for its own occupancy (a
  // whole number of resident rounds over (group, head) pairs), each split
  // holding <= 128 page items; fixed pages_per_split keeps the BEAM form
  bool use_beam4 = false;
  if (row_group == 4 && pps_fixed <= 0 && kv->kv_dtype == LLM_F16 && TS * D * 2 <= 8192 &&
      tn.beam4 && !tn.beam_mfma) {
    const long long groups = (long long)((B + 3) / 4) * H;
    const long long need = (4LL * ntiles_max + kMaxPps - 1) / kMaxPps;
    long long ns = (tune_beam4_resident_for(D, TS) + groups - 1) / groups;
    ns = std::max(std::max(ns, need), 2LL);
    ns = std::min(ns, max_nsplit(B, H, ntiles_max));
    if (tn.beam4_splits >= 2) ns = std::min<long long>(tn.beam4_splits, max_nsplit(B, H, ntiles_max));
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
  // beam groups of 4 fp16 rows with counters: dynamic tile assignment
  const bool steal_form = tn.beam_steal && row_group >= 4 && !direct &&
                          kv->kv_dtype == LLM_F16 && pps_fixed <= 0 && !use_beam4 &&
                          !tn.beam_mfma && steal_shape_ok(D, TS);
  if (plan) {
    const int group = std::max(1, std::min(row_group, 4));
    const bool wg = wgm_ok && !direct && group == 1 && nsplit <= kWgmMaxSplits;
    const bool beam = group == 4 && !direct && kv->kv_dtype == LLM_F16 &&
                      TS * D * 2 <= 8192;
    const bool steal = steal_form && rows && rows->beam_ctr;
    plan->nsplit = nsplit;
    plan->form = (direct ? LLM_PA_FORM_DIRECT : wg ? LLM_PA_FORM_WG_MERGE
                  : row_out ? LLM_PA_FORM_SPLIT_MERGE_ROW : LLM_PA_FORM_SPLIT_MERGE) |
                 (beam ? LLM_PA_FORM_BEAM : 0) | (oproj && wg ? LLM_PA_FORM_OPROJ : 0) |
                 (steal ? LLM_PA_FORM_STEAL : 0);
    return LLM_OK;
  }
  unsigned* steal_ctr = nullptr;
  if (steal_form)
    steal_ctr = rows && rows->beam_ctr ? rows->beam_ctr
                                       : tune_steal_counters(2 * (size_t)((B + 3) / 4) * H);
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
  a.balance16 = tn.beam_balance16;
  // beam-group workgroups in split-major order (PaSplitArgs::smaj).  Same box,
  // C4 (profiles/r06/c4_smaj_ab.txt): 12,719-12,737 against 12,604-12,617
  // tok/s; the launch's HBM bytes 1.031 -> 1.014x algorithmic
  // (profiles/pmc_attention_c4.json), the exits by dispatch slot unchanged
  a.smaj = a.group == 4 && tn.beam_smaj ? 1 : 0;
  a.beam4 = use_beam4 ? 1 : 0;
  a.steal = a.group == 4 ? steal_ctr : nullptr;
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
