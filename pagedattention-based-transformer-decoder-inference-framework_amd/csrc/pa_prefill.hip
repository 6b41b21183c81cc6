// Causal paged attention of a prompt chunk on MFMA (the reference's is_prefill
// pass: AttentionCUDA's `is_prefill` flag, attention/attention_cuda.hpp:21,
// with the maths of cpu_paged_attention_forward,
// attention_cpu/cpu_attention_kernel.cpp:37-129, per query token; SURVEY §8f
// row 4).
//
// m query tokens of ONE sequence sit at positions p0 .. p0+m-1 and their K/V
// are already in the sequence's pages (page-table row `row`).  Query i attends
// to positions 0 .. p0+i.  The decode kernel computes the same thing with one
// wave per (token, head), so each page is re-read once per query token; here a
// workgroup of NW waves owns 16·NW consecutive queries of one head, stages
// every 32-key block of K and V into LDS ONCE, and each wave runs
//   S^T[32 keys][16 queries] = K · Q^T        (v_mfma_f32_16x16x32_f16)
//   O^T[D][16 queries]     += V^T · P^T
// with the flash online softmax (log2 units, as pa_split_kernel) in between.
//
// Orientation: keys are the MFMA row index of S^T, so the C layout of S^T
// (lane l: rows 4(l>>4)+r, column l&15) already holds, per lane, 8 keys of ONE
// query: that is the B operand of the P·V product once the 32 keys are taken
// in the k order slot(key) = 8·((key&15)>>2) + 4·(key>>4) + (key&3).  V is
// staged row-major and its V^T A operand, in that same key order, is two
// hardware-transposed LDS reads (ds_read_b64_tr_b16) per 16 dims.  The query is the lane's column in both
// products, so the running max / sum / rescale are per lane (the 4 lanes of a
// query agree after a 2-step max exchange).
//
// Accuracy: q (fp32, pre-scaled by sm_scale·log2e) and p (fp32) are split into
// fp16 hi + lo halves and each product is two MFMAs; K and V are fp16 already.
// Both are first scaled by a power of two (q per query to |q|max ≈ 2^14, p by
// 2^14) because the MFMA drops fp16 subnormal inputs: unscaled, the lo half
// of every p < 0.25 was lost (1e-5 .. 5e-5 output error, measured).  Scaled,
// products of fp16 pairs are exact in the fp32 accumulator and the output
// error is at the decode kernel's level (scripts/diag_prefill.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "pa_decode.hpp"
#include "row_ops.hpp"

namespace llm {
namespace {

struct PaPrefillArgs {
  const float* q;
  int q_stride;  // floats between query rows
  float* out;
  int out_stride;
  const uint8_t* k_pool;
  const uint8_t* v_pool;
  size_t page_stride;     // bytes
  const int32_t* pt_row;  // page_table + row * H * max_tiles
  int H, max_tiles, num_pages;
  int p0, m;
  float qscale;  // sm_scale * log2(e)
  // key-range split (blockIdx.z = split s: tiles [s*pps, (s+1)*pps)); with
  // part_acc the unnormalised state goes to the decode layout
  // [(i*H + h)*nsplit + s][D] / [..][2] (m, l) for pa_merge_rows_internal
  int nsplit, pps;
  float* part_acc;
  float* part_ml;
};

constexpr int kKeyBlock = 32;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
constexpr float kPScale = 16384.f;  // P enters the PV MFMA as p * 2^14 (hi + lo)

__device__ __forceinline__ void split_f16(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

template <int D, int TS, int NW>
__global__ __launch_bounds__(64 * NW) void pa_prefill_kernel(PaPrefillArgs a) {
  constexpr int KB = kKeyBlock;
  constexpr int KSTR = D + 8;   // K row stride (halves): conflict-free 16-B row reads
  constexpr int VSTR = D + 16;  // V row stride (halves): 8·odd dwords, so the
                                // 64 lanes of a transposed read hit 64 banks
  constexpr int CPR = D / 8;    // 16-byte chunks per key row
  constexpr int NCH = KB * CPR; // chunks per block, each of K and V
  constexpr int NTH = 64 * NW;
  constexpr int CPT = NCH / NTH;
  constexpr int NKK = D / 32;   // k-steps of q.k
  constexpr int ND = D / 16;    // 16-dim tiles of the output
  static_assert(NCH % NTH == 0 && D % 32 == 0 && KB % TS == 0, "shape");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[KB * KSTR];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[KB * VSTR];
  __shared__ int kval[KB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = wave_id_uniform();
  const int g = lane >> 4;
  const int c = lane & 15;
  const int h = blockIdx.y;
  const int qbase = blockIdx.x * 16 * NW;
  const int qi = qbase + w * 16 + c;  // this lane's query (column of S^T / O^T)
  const int qpos = a.p0 + qi;
  const int lastpos = a.p0 + min(qbase + 16 * NW, a.m) - 1;  // last key any query here sees
  const int split = blockIdx.z;
  const int kb0 = split * a.pps * TS / KB;
  const int nblk = min((split + 1) * a.pps * TS / KB, lastpos / KB + 1);
  // no query of this workgroup reaches this split: the merge never reads it
  if (kb0 >= nblk) return;
  const int32_t* pt = a.pt_row + (size_t)h * a.max_tiles;

  // Q^T B-operand fragments: lane holds q[qi][32kk + 8g .. +7] (pre-scaled by
  // qscale), hi + lo.  The query's values are also scaled by a power of two
  // 2^(14-e) (|q|max < 2^e) so the lo halves stay clear of fp16 subnormals,
  // which the MFMA does not keep; S is scaled back exactly after the MFMA.
  float qx[NKK][8];
  float amax = 0.f;
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    f32x4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = x0;
    if (qi < a.m) {
      const float* qp = a.q + (size_t)qi * a.q_stride + h * D + 32 * kk + 8 * g;
      x0 = *reinterpret_cast<const f32x4*>(qp);
      x1 = *reinterpret_cast<const f32x4*>(qp + 4);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qx[kk][e] = x0[e] * a.qscale;
      qx[kk][4 + e] = x1[e] * a.qscale;
      amax = fmaxf(amax, fmaxf(fabsf(qx[kk][e]), fabsf(qx[kk][4 + e])));
    }
  }
  amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
  int qe = 0;
  (void)frexpf(amax, &qe);  // amax < 2^qe (0 for amax == 0)
  qe = min(max(qe, -100), 100);
  const float qsc = ldexpf(1.f, 14 - qe), qinv = ldexpf(1.f, qe - 14);
  f16x8 qh[NKK], ql[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      _Float16 hi, lo;
      split_f16(qx[kk][e] * qsc, hi, lo);
      qh[kk][e] = hi;
      ql[kk][e] = lo;
    }

  // Staging: chunk i of a thread = (key ch / CPR, dims 8 (ch % CPR)) of K and
  // of V — rows coalesced, both stored row-major ([key][d]); the PV product
  // reads V transposed with ds_read_b64_tr_b16.
  u32x4 kr[CPT], vr[CPT];
  int vok[CPT];
  auto page_of = [&](int kg) -> int {  // page of key position kg, -1 if none / past lastpos
    const int tile = kg / TS;
    int pg = (kg <= lastpos && tile < a.max_tiles) ? pt[tile] : -1;
    return (pg >= 0 && pg < a.num_pages) ? pg : -1;
  };
  auto load = [&](int kb) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int ch = tid + i * NTH;
      const int key = ch / CPR, d0 = (ch % CPR) * 8;
      const int kg = kb * KB + key;
      const int pg = page_of(kg);
      const size_t off = (size_t)pg * a.page_stride + ((kg % TS) * D + d0) * 2;
      vok[i] = pg >= 0;
      // masked keys stage V = 0: a never-written row may hold NaN (0 * NaN)
      kr[i] = pg >= 0 ? *reinterpret_cast<const u32x4*>(a.k_pool + off) : u32x4{0u, 0u, 0u, 0u};
      vr[i] = pg >= 0 ? *reinterpret_cast<const u32x4*>(a.v_pool + off) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int ch = tid + i * NTH;
      const int key = ch / CPR, d0 = (ch % CPR) * 8;
      *reinterpret_cast<u32x4*>(&Ks[key * KSTR + d0]) = kr[i];
      *reinterpret_cast<u32x4*>(&Vs[key * VSTR + d0]) = vr[i];
      if (d0 == 0) kval[key] = vok[i];
    }
  };

  f32x4 O[ND];
#pragma unroll
  for (int nd = 0; nd < ND; ++nd) O[nd] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun = kNegSentinel, lrun = 0.f;

  load(kb0);
  for (int kb = kb0; kb < nblk; ++kb) {
    if (kb > kb0) __syncthreads();  // every wave is done reading block kb-1
    stage();
    __syncthreads();
    if (kb + 1 < nblk) load(kb + 1);  // next block's loads fly during this block's math

    // S^T: two 16-key tiles
    f32x4 s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(&Ks[(16 * t + c) * KSTR + 32 * kk + 8 * g]);
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qh[kk], s[t], 0, 0, 0);
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, ql[kk], s[t], 0, 0, 0);
      }
      s[t] *= qinv;
    }
    // causal + missing-page mask, online softmax (per query = per lane)
    bool ok[2][4];
    float mloc = kNegSentinel;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * t + 4 * g + r;
        ok[t][r] = kval[key] != 0 && kb * KB + key <= qpos;
        if (ok[t][r]) mloc = fmaxf(mloc, s[t][r]);
      }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mnew = fmaxf(mrun, mloc);
    const float corr = __builtin_amdgcn_exp2f(mrun - mnew);
    lrun *= corr;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) O[nd] *= corr;
    f16x8 ph, pl;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = ok[t][r] ? __builtin_amdgcn_exp2f(s[t][r] - mnew) : 0.f;
        lrun += p;
        _Float16 hi, lo;
        split_f16(p * kPScale, hi, lo);  // p <= 1: scaled clear of fp16 subnormals
        ph[4 * t + r] = hi;
        pl[4 * t + r] = lo;
      }
    mrun = mnew;
    // O^T += V^T · P^T.  A operand lane l: V^T[d = 16nd + (l&15)][k 8g+j] =
    // V[key(8g+j)][d], keys 4g..4g+3 then 16+4g..16+4g+3: two transposed
    // reads of 4 V rows x 16 columns, lane 4q+p addressing row q, columns 4p..
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const int q4 = c >> 2, p4 = c & 3;
      const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)&Vs[(4 * g + q4) * VSTR + 16 * nd + 4 * p4]);
      const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)&Vs[(16 + 4 * g + q4) * VSTR + 16 * nd + 4 * p4]);
      const f16x8 vf = __builtin_bit_cast(
          f16x8, s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
      O[nd] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, ph, O[nd], 0, 0, 0);
      O[nd] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pl, O[nd], 0, 0, 0);
    }
  }

  // the 4 lanes of a query hold partial sums over their keys
  lrun += __shfl_xor(lrun, 16, 64);
  lrun += __shfl_xor(lrun, 32, 64);
  if (qi < a.m) {
    if (a.part_acc) {  // split partial state (unnormalised, log2 units)
      const size_t pidx = ((size_t)qi * a.H + h) * a.nsplit + split;
      float* o = a.part_acc + pidx * D + 4 * g;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) *reinterpret_cast<f32x4*>(o + 16 * nd) = O[nd] * (1.0f / kPScale);
      if (g == 0) *reinterpret_cast<float2*>(a.part_ml + pidx * 2) = float2{mrun, lrun};
    } else {
      const float inv = 1.0f / (lrun + 1e-6f) * (1.0f / kPScale);
      float* o = a.out + (size_t)qi * a.out_stride + h * D + 4 * g;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) *reinterpret_cast<f32x4*>(o + 16 * nd) = O[nd] * inv;
    }
  }
}

template <int D, int TS>
hipError_t launch_prefill(const PaPrefillArgs& a, int nw, hipStream_t st) {
  if (nw == 4) {
    const dim3 grid((a.m + 63) / 64, a.H, a.nsplit);
    hipLaunchKernelGGL((pa_prefill_kernel<D, TS, 4>), grid, dim3(256), 0, st, a);
  } else {
    const dim3 grid((a.m + 31) / 32, a.H, a.nsplit);
    hipLaunchKernelGGL((pa_prefill_kernel<D, TS, 2>), grid, dim3(128), 0, st, a);
  }
  return hipGetLastError();
}

// Launch geometry: NW waves (16 queries each) per workgroup; the key range is
// split until the grid holds about kTargetWgs workgroups (4 per CU), in
// splits of whole 32-key blocks and at least 2 blocks each.
constexpr int kTargetWgs = 1024;
struct PrefillPlan {
  int nw, nsplit, pps;
};
PrefillPlan prefill_plan(const pa_kv_view* kv, int p0, int m) {
  PrefillPlan p;
#if LLM_TUNING
  p.nw = env_int("LLM_PREFILL_NW", 4) == 2 ? 2 : 4;
#else
  p.nw = 4;
#endif
  const int TS = kv->page_size;
  const int step = kKeyBlock / TS;  // tiles per key block
  const int ntiles = (p0 + m + TS - 1) / TS;
  const int nq = (m + 16 * p.nw - 1) / (16 * p.nw);
  const int want = std::min(std::max(kTargetWgs / std::max(nq * kv->num_heads, 1), 1), 128);
  int pps = (ntiles + want - 1) / want;
  pps = std::max((pps + step - 1) / step * step, 2 * step);
  p.pps = pps;
  p.nsplit = std::max(1, std::min((ntiles + pps - 1) / pps, 128));
  if (p.nsplit * pps < ntiles) {  // > 128 splits: lengthen them
    p.pps = ((ntiles + 127) / 128 + step - 1) / step * step;
    p.nsplit = (ntiles + p.pps - 1) / p.pps;
  }
  return p;
}

}  // namespace

bool pa_prefill_supported(const pa_kv_view* kv) {
  return kv && kv->kv_dtype == LLM_F16 && (kv->head_dim == 64 || kv->head_dim == 128) &&
         (kv->page_size == 16 || kv->page_size == 32);
}

size_t pa_prefill_ws_bytes(const pa_kv_view* kv, int p0, int m) {
  if (!pa_prefill_supported(kv) || m <= 0 || p0 < 0) return 0;
  const PrefillPlan p = prefill_plan(kv, p0, m);
  if (p.nsplit <= 1) return 0;
  return (size_t)m * kv->num_heads * p.nsplit * (size_t)(kv->head_dim + 2) * sizeof(float);
}

int pa_prefill_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                        int out_stride, int row, int p0, int m, float sm_scale, void* workspace,
                        size_t workspace_bytes, hipStream_t st, const PaRowOutputs* rows) {
  LLM_REQUIRE(kv && q, "pa_prefill: NULL argument");
  if (!pa_prefill_supported(kv))
    return fail(LLM_ERR_UNSUPPORTED,
                "pa_prefill: fp16 pools with head_dim 64 or 128 and page_size 16 or 32 only");
  const int H = kv->num_heads, D = kv->head_dim, hid = H * D;
  LLM_REQUIRE(m >= 1 && p0 >= 0, "pa_prefill: need m >= 1 and p0 >= 0");
  LLM_REQUIRE(row >= 0 && row < kv->num_beams, "pa_prefill: row outside the page table");
  LLM_REQUIRE((long long)(p0 + m + kv->page_size - 1) / kv->page_size <= kv->max_tiles,
              "pa_prefill: positions past the page table's max_tiles");
  if (q_stride <= 0) q_stride = hid;
  if (out_stride <= 0) out_stride = hid;
  LLM_REQUIRE(q_stride >= hid && out_stride >= hid && q_stride % 4 == 0 && out_stride % 4 == 0,
              "pa_prefill: row strides must be >= H*D and multiples of 4");
  LLM_REQUIRE(reinterpret_cast<uintptr_t>(q) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0,
              "pa_prefill: q and out must be 16-byte aligned");
  const bool row_out = rows && (rows->q || rows->out16);
  PrefillPlan pl = prefill_plan(kv, p0, m);
  const size_t need = pa_prefill_ws_bytes(kv, p0, m);
  const bool split = pl.nsplit > 1 && workspace && workspace_bytes >= need &&
                     (out == nullptr || out_stride == hid) &&
                     (!row_out || rows->pack);  // the merge writes packed o_proj inputs
  LLM_REQUIRE(out || (split && row_out), "pa_prefill: out is NULL");
  PaPrefillArgs a{};
  a.q = q;
  a.q_stride = q_stride;
  a.out = out;
  a.out_stride = out_stride;
  a.k_pool = static_cast<const uint8_t*>(kv->k_pool);
  a.v_pool = static_cast<const uint8_t*>(kv->v_pool);
  a.page_stride = kv_view_page_stride(*kv);
  a.pt_row = kv->page_table + (size_t)row * H * kv->max_tiles;
  a.H = H;
  a.max_tiles = kv->max_tiles;
  a.num_pages = kv->num_pages;
  a.p0 = p0;
  a.m = m;
  a.qscale = sm_scale * kLog2e;
  if (split) {
    a.nsplit = pl.nsplit;
    a.pps = pl.pps;
    a.part_acc = static_cast<float*>(workspace);
    a.part_ml = a.part_acc + (size_t)m * H * pl.nsplit * D;
  } else {
    a.nsplit = 1;
    a.pps = kv->max_tiles;
  }
  hipError_t e;
  const int TS = kv->page_size;
  if (D == 64)
    e = TS == 16 ? launch_prefill<64, 16>(a, pl.nw, st) : launch_prefill<64, 32>(a, pl.nw, st);
  else
    e = TS == 16 ? launch_prefill<128, 16>(a, pl.nw, st) : launch_prefill<128, 32>(a, pl.nw, st);
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("pa_prefill launch: ") + hipGetErrorString(e));
  if (split)
    return pa_merge_rows_internal(a.part_acc, a.part_ml, (rows && !rows->keep_out) ? nullptr : out,
                                  rows, nullptr, p0, m, H, D, p0 + m, TS, pl.pps, pl.nsplit,
                                  kv->max_tiles, st);
  if (row_out) {  // one pass: convert the fp32 rows into the o_proj input
    if (rows->q)
      LLM_HIP_RET(launch_quantize_rows(out, m, hid, rows->q, rows->inv_scale, st, rows->pack));
    if (rows->out16)
      LLM_HIP_RET(launch_to_f16(out, (size_t)m * hid, rows->out16, st, rows->pack ? hid : 0));
  }
  return LLM_OK;
}

}  // namespace llm

extern "C" size_t pa_prefill_workspace_bytes(const pa_kv_view* kv, int p0, int m) {
  return llm::pa_prefill_ws_bytes(kv, p0, m);
}

extern "C" int pa_prefill(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                          int out_stride, int row, int p0, int m, float sm_scale, void* workspace,
                          size_t workspace_bytes, void* stream) {
  LLM_REQUIRE(out, "pa_prefill: out is NULL");
  return llm::pa_prefill_internal(kv, q, q_stride, out, out_stride, row, p0, m, sm_scale,
                                  workspace, workspace_bytes, llm::as_stream(stream));
}
