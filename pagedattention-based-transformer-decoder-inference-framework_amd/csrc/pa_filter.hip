// Paged attention with the reference's optional stages: top-k / top-p / EOS
// filtering of the attention weights and the attention-weight / score outputs.
//
// This is the full contract of cpu_paged_attention_forward
// (attention_cpu/cpu_attention_kernel.cpp:37-129) and its input/output structs
// CPUAttentionInput / CPUAttentionOutput (attention_cpu/attention_cpu.hpp:8-43:
// temperature, top_k, top_p, eos_token, eos_threshold; attention_weights,
// logits), which the GPU kernel of the reference tries to offer through its
// top_k / top_p / rerank_scores arguments
// (attention/paged_flash_attention_kernel_fused.cu:5-90, broken: Appendix A #2,
// #5).  The hot decode path never enables these stages (pa_decode.hip); this
// kernel runs when a caller asks for them.
//
// One workgroup per (row b, head h).  The whole row of scores lives in LDS
// (T <= 8192), or, for longer rows, in the caller's workspace (the row's
// scores and sort keys, pa_decode_ex_workspace_bytes; only its own workgroup
// touches them, so the barriers that order the LDS form order these too):
// scores -> softmax -> (sort by (prob, index) descending ->
// top-k / top-p mask) -> EOS threshold -> AV.  The sort key is
// (prob bits << 32 | index): probabilities are >= 0, so the unsigned order of
// the key is exactly std::greater on pair<float, int> — the order
// apply_topk_topp_filter sorts by (attention_cpu/softmax_lut.cpp:233-256),
// ties broken toward the larger index.
#include "common.hpp"
#include "pa_decode.hpp"

#include <algorithm>

#include <string>

namespace llm {

constexpr int kFilterThreads = 1024;
constexpr int kFilterMaxT = 8192;

struct PaFilterArgs {
  const uint8_t* k_pool;
  const uint8_t* v_pool;
  const int32_t* page_table;
  const float* q;
  float* out;         // [B][H][D]
  float* probs_out;   // [B][H][T] or null
  float* scores_out;  // [B][H][T] or null
  const int32_t* beam_ids;
  const int32_t* context_lens;
  int B, H, D, T, TS;
  int num_pages, num_beams, max_tiles;
  size_t page_stride;  // elements from page p to page p + 1
  float temperature;
  uint64_t* ws_key;   // [B*H][Tp] sort keys (the workspace form)
  float* ws_sc;       // [B*H][Tp] scores / probabilities (the workspace form)
  int Tp;             // row stride of ws_key / ws_sc
  int top_k;
  float top_p;
  int eos;
  float eos_thr;
};

template <int KVT>
__device__ __forceinline__ float kv_elem(const uint8_t* pool, size_t i) {
  if constexpr (KVT == LLM_F16) {
    return (float)reinterpret_cast<const _Float16*>(pool)[i];
  } else if constexpr (KVT == LLM_BF16) {
    return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(pool)[i] << 16);
  } else if constexpr (KVT == LLM_F32) {
    return reinterpret_cast<const float*>(pool)[i];
  } else {
    return (float)reinterpret_cast<const int8_t*>(pool)[i];
  }
}

// Block-wide reduction of one value per thread (all threads get the result).
template <bool MAX>
__device__ float block_reduce(float x, float* sh) {
  x = MAX ? wave_max(x) : wave_sum(x);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = x;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < kFilterThreads / 64; ++i) r = MAX ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

template <int KVT, bool WS>
__global__ __launch_bounds__(kFilterThreads) void pa_filter_kernel(PaFilterArgs a) {
  __shared__ float qs[256];
  __shared__ float lsc[WS ? 1 : kFilterMaxT];  // scores, then probabilities
  __shared__ uint64_t lkey[WS ? kFilterThreads / 2 : kFilterMaxT];  // WS: the AV reduction only
  __shared__ float sh[kFilterThreads / 64];
  const int tid = threadIdx.x;
  const int bh = blockIdx.x;
  float* sc = WS ? a.ws_sc + (size_t)bh * a.Tp : lsc;
  uint64_t* key = WS ? a.ws_key + (size_t)bh * a.Tp : lkey;
  const int b = bh / a.H, h = bh % a.H;
  const int D = a.D;
  const int r = a.beam_ids ? a.beam_ids[b] : b;
  int Tb = a.context_lens ? a.context_lens[b] : a.T;
  Tb = min(max(Tb, 0), a.T);
  const bool row_ok = r >= 0 && r < a.num_beams;
  const int32_t* table = a.page_table + ((size_t)(row_ok ? r : 0) * a.H + h) * a.max_tiles;
  auto page_of = [&](int t) -> int {  // KVTileCache::get (kv_tile_cache.hpp:21-26)
    const int tile = t / a.TS;
    if (!row_ok || tile >= a.max_tiles) return -1;
    const int p = table[tile];
    return (p < 0 || p >= a.num_pages) ? -1 : p;
  };
  for (int d = tid; d < D; d += kFilterThreads) qs[d] = a.q[(size_t)bh * D + d];
  __syncthreads();

  // scores[t] = dot(q, k_t) / temperature; -1e9 where the tile is missing
  // (cpu_attention_kernel.cpp:61,68-86)
  for (int t = tid; t < Tb; t += kFilterThreads) {
    const int p = page_of(t);
    float s = -1e9f;
    if (p >= 0) {
      const size_t base = (size_t)p * a.page_stride + (size_t)(t % a.TS) * D;
      float dot = 0.f;
      for (int d = 0; d < D; ++d) dot += qs[d] * kv_elem<KVT>(a.k_pool, base + d);
      s = dot / a.temperature;
    }
    sc[t] = s;
  }
  __syncthreads();
  if (a.scores_out)
    for (int t = tid; t < a.T; t += kFilterThreads)
      a.scores_out[(size_t)bh * a.T + t] = t < Tb ? sc[t] : -1e9f;

  // softmax_lut_vec (softmax_lut.cpp:203-231): exp((s - max) / temperature) / (sum + 1e-6)
  float mx = -1e9f;
  for (int t = tid; t < Tb; t += kFilterThreads) mx = fmaxf(mx, sc[t]);
  mx = block_reduce<true>(mx, sh);
  float sum = 0.f;
  for (int t = tid; t < Tb; t += kFilterThreads) {
    const float e = expf((sc[t] - mx) / a.temperature);
    sc[t] = e;
    sum += e;
  }
  sum = block_reduce<false>(sum, sh);
  const float inv = 1.0f / (sum + 1e-6f);
  for (int t = tid; t < Tb; t += kFilterThreads) sc[t] = sc[t] * inv;
  __syncthreads();

  // apply_topk_topp_filter (softmax_lut.cpp:233-256): rank by (prob, index)
  // descending; zero rank >= top_k and every entry whose preceding mass
  // (cum of the higher-ranked probabilities) is >= top_p; no renormalisation.
  if ((a.top_k > 0 || a.top_p < 1.0f) && Tb > 0) {
    int Tp = 1;
    while (Tp < Tb) Tp <<= 1;
    for (int i = tid; i < Tp; i += kFilterThreads)
      key[i] = i < Tb ? ((uint64_t)__float_as_uint(sc[i]) << 32) | (uint32_t)i : 0ull;
    __syncthreads();
    for (int k = 2; k <= Tp; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < Tp; i += kFilterThreads) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const uint64_t x = key[i], y = key[ixj];
            const bool desc = (i & k) == 0;
            if (desc ? x < y : x > y) {
              key[i] = y;
              key[ixj] = x;
            }
          }
        }
        __syncthreads();
      }
    // exclusive prefix of the sorted probabilities: each thread owns E
    // consecutive ranks, then a block scan of the per-thread totals
    const int E = (Tp + kFilterThreads - 1) / kFilterThreads;
    const int i0 = tid * E;
    float part = 0.f;
    for (int e = 0; e < E; ++e)
      if (i0 + e < Tb) part += __uint_as_float((uint32_t)(key[i0 + e] >> 32));
    float incl = part;
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    __syncthreads();
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    float before = incl - part;
    for (int i = 0; i < w; ++i) before += sh[i];
    float cum = before;
    for (int e = 0; e < E; ++e) {
      const int i = i0 + e;
      if (i >= Tb) break;
      const uint64_t kv = key[i];
      if ((a.top_k > 0 && i >= a.top_k) || (a.top_p < 1.0f && cum >= a.top_p))
        sc[(uint32_t)kv] = 0.f;
      cum += __uint_as_float((uint32_t)(kv >> 32));
    }
    __syncthreads();
  }
  // EOS hard threshold: keep only the EOS position when its weight exceeds it
  if (a.eos >= 0 && a.eos < Tb && sc[a.eos] > a.eos_thr) {
    const int eos = a.eos;
    __syncthreads();
    for (int t = tid; t < Tb; t += kFilterThreads)
      if (t != eos) sc[t] = 0.f;
    __syncthreads();
  }
  if (a.probs_out)
    for (int t = tid; t < a.T; t += kFilterThreads)
      a.probs_out[(size_t)bh * a.T + t] = t < Tb ? sc[t] : 0.f;

  // out = sum_t p_t v_t over present tiles (cpu_attention_kernel.cpp:103-117):
  // thread -> (dim d, token group g), groups summed in order at the end
  const int G = kFilterThreads / D;
  const int d = tid % D, g = tid / D;
  float acc = 0.f;
  if (g < G)
    for (int t = g; t < Tb; t += G) {
      const float p = sc[t];
      if (p == 0.f) continue;
      const int pg = page_of(t);
      if (pg < 0) continue;
      acc += p * kv_elem<KVT>(a.v_pool, (size_t)pg * a.page_stride + (size_t)(t % a.TS) * D + d);
    }
  float* red = reinterpret_cast<float*>(lkey);
  __syncthreads();
  if (g < G) red[g * D + d] = acc;
  __syncthreads();
  if (tid < D) {
    float o = 0.f;
    for (int gg = 0; gg < G; ++gg) o += red[gg * D + tid];
    a.out[(size_t)bh * D + tid] = o;
  }
}

}  // namespace llm

using namespace llm;

namespace {
// The longest row the filtered form takes: its power-of-two sort length must
// stay an int (filter_row_stride), and 2^30 tokens is far past any context
constexpr int kFilterRowMaxT = 1 << 30;
int filter_row_stride(int T) {  // the bitonic sort's power-of-two length, T <= kFilterRowMaxT
  int Tp = 1;
  while (Tp < T) Tp <<= 1;
  return Tp;
}
}  // namespace

extern "C" size_t pa_decode_ex_workspace_bytes(int B, int H, int T) {
  if (B <= 0 || H <= 0 || T <= kFilterMaxT || T > kFilterRowMaxT) return 0;
  return (size_t)B * H * filter_row_stride(T) * (sizeof(uint64_t) + sizeof(float));
}

extern "C" int pa_decode_ex(const pa_kv_view* kv, const float* q, float* out,
                            const int32_t* beam_ids, const int32_t* context_lens, int B, int H,
                            int D, int T, const pa_decode_options* opt, void* workspace,
                            size_t workspace_bytes, void* stream) {
  LLM_REQUIRE(kv != nullptr && opt != nullptr, "pa_decode_ex: kv / opt is NULL");
  LLM_REQUIRE(B >= 0 && H > 0 && D > 0 && T >= 0, "pa_decode_ex: bad B/H/D/T");
  LLM_REQUIRE(opt->temperature > 0.f, "pa_decode_ex: temperature must be > 0");
  const bool filtered = opt->top_k > 0 || opt->top_p < 1.0f || opt->eos_token >= 0 ||
                        opt->probs_out || opt->scores_out;
  if (!filtered) {
    // the hot path: identical maths with sm_scale = 1 / temperature^2 (Appendix A #13)
    return pa_decode(kv, q, out, beam_ids, context_lens, B, H, D, T,
                     1.0f / (opt->temperature * opt->temperature), 0, workspace,
                     workspace_bytes, stream);
  }
  if (B == 0) return LLM_OK;
  LLM_REQUIRE(q && out && kv->k_pool && kv->v_pool && kv->page_table, "pa_decode_ex: NULL pointer");
  LLM_REQUIRE(kv->num_heads == H && kv->head_dim == D, "pa_decode_ex: H/D differ from the kv view");
  LLM_REQUIRE(kv->page_size > 0 && kv->num_pages > 0 && kv->num_beams > 0 && kv->max_tiles > 0,
              "pa_decode_ex: empty kv view");
  LLM_REQUIRE(opt->top_p > 0.f, "pa_decode_ex: top_p must be > 0");
  LLM_REQUIRE(kv->page_stride == 0 ||
                  (kv->page_stride >= (int64_t)kv->page_size * kv->head_dim *
                                          kv_elem_size(kv->kv_dtype) &&
                   kv->page_stride % 16 == 0),
              "pa_decode_ex: page_stride must be 0 or >= one page and a multiple of 16");
  if (D > 256) return fail(LLM_ERR_UNSUPPORTED, "pa_decode_ex: filters / weight outputs need D <= 256");
  if (T > kFilterRowMaxT)
    return fail(LLM_ERR_UNSUPPORTED, "pa_decode_ex: filters / weight outputs need T <= 2^30");
  const bool ws_form = T > kFilterMaxT;
  const size_t need = pa_decode_ex_workspace_bytes(B, H, T);
  LLM_REQUIRE(!ws_form || (workspace != nullptr && workspace_bytes >= need &&
                           reinterpret_cast<uintptr_t>(workspace) % 8 == 0),
              "pa_decode_ex: T > 8192 with filters needs an 8-byte aligned workspace of "
              "pa_decode_ex_workspace_bytes(B, H, T)");
  PaFilterArgs a{};
  a.k_pool = static_cast<const uint8_t*>(kv->k_pool);
  a.v_pool = static_cast<const uint8_t*>(kv->v_pool);
  a.page_table = kv->page_table;
  a.q = q;
  a.out = out;
  a.probs_out = opt->probs_out;
  a.scores_out = opt->scores_out;
  a.beam_ids = beam_ids;
  a.context_lens = context_lens;
  a.B = B; a.H = H; a.D = D; a.T = T; a.TS = kv->page_size;
  a.num_pages = kv->num_pages; a.num_beams = kv->num_beams; a.max_tiles = kv->max_tiles;
  a.page_stride = kv_view_page_stride(*kv) / std::max(1, kv_elem_size(kv->kv_dtype));
  a.temperature = opt->temperature;
  if (ws_form) {
    a.Tp = filter_row_stride(T);
    a.ws_key = static_cast<uint64_t*>(workspace);
    a.ws_sc = reinterpret_cast<float*>(a.ws_key + (size_t)B * H * a.Tp);
  }
  a.top_k = opt->top_k;
  a.top_p = opt->top_p;
  a.eos = opt->eos_token;
  a.eos_thr = opt->eos_threshold;
  hipStream_t st = as_stream(stream);
  const dim3 grid(B * H), block(kFilterThreads);
#define LLM_FILTER_LAUNCH(KVT)                                                  \
  do {                                                                          \
    if (ws_form)                                                                \
      hipLaunchKernelGGL((pa_filter_kernel<KVT, true>), grid, block, 0, st, a);  \
    else                                                                        \
      hipLaunchKernelGGL((pa_filter_kernel<KVT, false>), grid, block, 0, st, a); \
  } while (0)
  switch (kv->kv_dtype) {
    case LLM_F16: LLM_FILTER_LAUNCH(LLM_F16); break;
    case LLM_BF16: LLM_FILTER_LAUNCH(LLM_BF16); break;
    case LLM_F32: LLM_FILTER_LAUNCH(LLM_F32); break;
    case LLM_I8: LLM_FILTER_LAUNCH(LLM_I8); break;
    default: return fail(LLM_ERR_INVALID, "pa_decode_ex: kv_dtype");
  }
#undef LLM_FILTER_LAUNCH
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}
