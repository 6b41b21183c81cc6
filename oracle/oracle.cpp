// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's paged-attention decode path and of the
// INT8Decoder layer maths.  Only tests/, bench.py's
// cpu_baseline leg and __graft_entry__.smoke() may load this library, and only
// as the checker / CPU baseline.  The product path (the HIP library under
// pagedattention-based-transformer-decoder-inference-framework_amd/csrc) never
// links or calls it.
//
// Parity pinning: the attention / softmax / quantizer / LayerNorm / MLP pieces
// below are checked against golden vectors produced by
// oracle/ref_golden/gen_golden.cpp, which links the reference's own compilable
// sources (kv_tile_cache_cpu.cpp, softmax_lut.cpp, int8_quant.cpp, mlp.hpp,
// layer_norm.hpp) — see tests/test_oracle_golden.py.  The INT8 GEMM contract
// (oneDNN, not vendored) is "parity unpinned" beyond the exact int32
// accumulator, which is cross-checked against torch._int_mm.
//
// Reference citations are relative to the reference tree root.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <utility>
#include <vector>
#include <omp.h>

namespace {

// Exact IEEE binary16 -> binary32 (no F16C dependency).
inline float half_to_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1Fu;
  uint32_t mant = h & 0x3FFu;
  uint32_t bits;
  if (exp == 0) {
    if (mant == 0) {
      bits = sign;
    } else {  // subnormal: renormalise
      exp = 127 - 15 + 1;
      while ((mant & 0x400u) == 0) { mant <<= 1; --exp; }
      mant &= 0x3FFu;
      bits = sign | (exp << 23) | (mant << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (mant << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (mant << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

// binary32 -> binary16, round to nearest even (matches __float2half_rn and
// numpy.float16).
inline uint16_t float_to_half(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t absx = x & 0x7FFFFFFFu;
  if (absx >= 0x7F800000u) {  // inf / nan
    return (uint16_t)(sign | 0x7C00u | (absx > 0x7F800000u ? 0x200u : 0));
  }
  if (absx >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);  // overflow -> inf
  if (absx < 0x33000001u) return (uint16_t)sign;                // underflow -> 0
  int e = (int)(absx >> 23) - 127;
  uint32_t m = (absx & 0x7FFFFFu) | 0x800000u;
  if (e < -14) {  // subnormal half
    const int shift = -14 - e + 13;
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1);
    const uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (r & 1u))) ++r;
    return (uint16_t)(sign | r);
  }
  uint32_t r = m >> 13;
  const uint32_t rem = m & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) ++r;
  uint32_t he = (uint32_t)(e + 15);
  if (r & 0x800u) { r >>= 1; ++he; }
  if (he >= 31) return (uint16_t)(sign | 0x7C00u);
  return (uint16_t)(sign | (he << 10) | (r & 0x3FFu));
}

// softmax_lut_vec restated (attention_cpu/softmax_lut.cpp:203-231): max over
// the scores, x = (s - max) / temperature, exp, block-of-8 partial sums, then
// multiply by 1 / (sum + 1e-6).  The reference requires len % 8 == 0; the
// restatement also handles a ragged tail the same way (blocks of up to 8).
void softmax_vec(const float* scores, int len, float temperature, float* out) {
  float maxval = -1e9f;
  for (int i = 0; i < len; ++i) maxval = std::max(maxval, scores[i]);
  float sum = 0.0f;
  for (int i = 0; i < len; i += 8) {
    float blk = 0.0f;
    const int n = std::min(8, len - i);
    for (int j = 0; j < n; ++j) {
      const float x = std::exp((scores[i + j] - maxval) / temperature);
      out[i + j] = x;
      blk += x;
    }
    sum += blk;
  }
  const float inv = 1.0f / (sum + 1e-6f);
  for (int i = 0; i < len; ++i) out[i] = out[i] * inv;
}

// apply_topk_topp_filter restated (attention_cpu/softmax_lut.cpp:233-256):
// stable descending sort of (prob, index), zero everything past top_k or past
// cumulative top_p, no renormalisation; optional EOS hard threshold.
void topk_topp_filter(float* probs, int len, int top_k, float top_p, int eos, float eos_thr) {
  if (top_k <= 0 && top_p >= 1.0f && eos < 0) return;
  std::vector<std::pair<float, int>> sorted;
  sorted.reserve(len);
  for (int i = 0; i < len; ++i) sorted.emplace_back(probs[i], i);
  std::sort(sorted.begin(), sorted.end(), std::greater<>());
  float cum = 0.0f;
  for (int i = 0; i < len; ++i) {
    const int idx = sorted[i].second;
    if ((top_k > 0 && i >= top_k) || (top_p < 1.0f && cum >= top_p)) probs[idx] = 0.0f;
    cum += sorted[i].first;
  }
  if (eos >= 0 && eos < len && probs[eos] > eos_thr)
    for (int i = 0; i < len; ++i)
      if (i != eos) probs[i] = 0.0f;
}

}  // namespace

extern "C" {

int oracle_version() { return 1; }

void oracle_half_to_float(const uint16_t* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = half_to_float(in[i]);
}

void oracle_float_to_half(const float* in, uint16_t* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = float_to_half(in[i]);
}

// PageTable::index / lookup restated (kv_cache/page_table.hpp:39-49):
// idx = beam * (H * NT) + head * NT + tile; out of range -> -1.
int oracle_page_lookup(const int32_t* table, int num_beams, int num_heads, int num_tiles,
                       int beam, int head, int tile) {
  const int64_t total = (int64_t)num_beams * num_heads * num_tiles;
  const int64_t idx = (int64_t)beam * (num_heads * num_tiles) + (int64_t)head * num_tiles + tile;
  if (idx < 0 || idx >= total) return -1;
  if (tile < 0 || tile >= num_tiles || head < 0 || head >= num_heads) return -1;
  return table[idx];
}

// cpu_paged_attention_forward restated (attention_cpu/cpu_attention_kernel.cpp:37-129).
//   * beam routing: beam = beam_ids ? beam_ids[b] : b                    (:50)
//   * scores[T] initialised to -1e9                                       (:61)
//   * tile walk, missing tile skipped, partial last tile                  (:68-86)
//   * score = dot(q, k_t) / temperature, decode query sees all keys       (:85; Appendix A #12)
//   * softmax_lut_vec (divides by temperature again)                      (softmax_lut.cpp:203-231)
//   * apply_topk_topp_filter                                              (softmax_lut.cpp:233-256)
//   * out = sum_t p_t v_t over present tiles                              (:103-117)
// KVTileCache<T>::get (kv_cache/kv_tile_cache.hpp:21-26): page < 0 or
// page >= num_pages -> no tile; else pool + page * ts * D.
// context_lens (nullable) gives a per-row T_b <= T (ragged batches).
int oracle_paged_attention(const float* q, const float* k_pool, const float* v_pool,
                           const int32_t* page_table, int num_pages, int ts, int num_beams,
                           int max_tiles, const int32_t* beam_ids, const int32_t* context_lens,
                           int B, int H, int D, int T, float temperature, int top_k, float top_p,
                           int eos_token, float eos_threshold, float* out, float* probs_out,
                           float* scores_out) {
  if (B < 0 || H <= 0 || D <= 0 || T < 0 || ts <= 0) return 1;
#pragma omp parallel for collapse(2) schedule(dynamic)
  for (int b = 0; b < B; ++b) {
    for (int h = 0; h < H; ++h) {
      const int beam = beam_ids ? beam_ids[b] : b;
      const int Tb = context_lens ? std::min(context_lens[b], T) : T;
      const int ntiles = (Tb + ts - 1) / ts;
      const float* qv = q + ((int64_t)b * H + h) * D;
      std::vector<float> scores(std::max(Tb, 1), -1e9f);
      std::vector<float> probs(std::max(Tb, 1), 0.0f);
      std::vector<const float*> ktile(ntiles, nullptr), vtile(ntiles, nullptr);
      for (int tile = 0; tile < ntiles; ++tile) {
        const int page = oracle_page_lookup(page_table, num_beams, H, max_tiles, beam, h, tile);
        if (page < 0 || page >= num_pages) continue;
        ktile[tile] = k_pool + (int64_t)page * ts * D;
        vtile[tile] = v_pool + (int64_t)page * ts * D;
      }
      for (int tile = 0; tile < ntiles; ++tile) {
        const int start = tile * ts;
        const int len = std::min(ts, Tb - start);
        const float* kt = ktile[tile];
        if (!kt) continue;
        for (int t = 0; t < len; ++t) {
          float dot = 0.0f;
          for (int d = 0; d < D; ++d) dot += qv[d] * kt[(int64_t)t * D + d];
          scores[start + t] = dot / temperature;
        }
      }
      float* o = out + ((int64_t)b * H + h) * D;
      for (int d = 0; d < D; ++d) o[d] = 0.0f;
      if (Tb > 0) {
        softmax_vec(scores.data(), Tb, temperature, probs.data());
        topk_topp_filter(probs.data(), Tb, top_k, top_p, eos_token, eos_threshold);
        for (int tile = 0; tile < ntiles; ++tile) {
          const int start = tile * ts;
          const int len = std::min(ts, Tb - start);
          const float* vt = vtile[tile];
          if (!vt) continue;
          for (int t = 0; t < len; ++t) {
            const float p = probs[start + t];
            for (int d = 0; d < D; ++d) o[d] += p * vt[(int64_t)t * D + d];
          }
        }
      }
      if (probs_out) {
        float* po = probs_out + ((int64_t)b * H + h) * T;
        for (int t = 0; t < T; ++t) po[t] = t < Tb ? probs[t] : 0.0f;
      }
      if (scores_out) {
        float* so = scores_out + ((int64_t)b * H + h) * T;
        for (int t = 0; t < T; ++t) so[t] = t < Tb ? scores[t] : -1e9f;
      }
    }
  }
  return 0;
}

// compute_minmax_scale (attention_cpu/int8_quant.cpp:59-64):
// scale = 127 / (max(|min|, |max|) + 1e-6).
float oracle_minmax_scale(const float* x, int64_t n) {
  float mn = x[0], mx = x[0];
  for (int64_t i = 1; i < n; ++i) { mn = std::min(mn, x[i]); mx = std::max(mx, x[i]); }
  const float absmax = std::max(std::fabs(mn), std::fabs(mx));
  return 127.f / (absmax + 1e-6f);
}

// quantize_to_int8 (attention_cpu/int8_quant.cpp:5-13): q = clamp(round(x*scale)).
void oracle_quantize(const float* x, int64_t n, float scale, int8_t* q) {
  for (int64_t i = 0; i < n; ++i) {
    int32_t v = (int32_t)std::round(x[i] * scale);
    v = std::max(-128, std::min(127, v));
    q[i] = (int8_t)v;
  }
}

// Per-row dynamic activation quantisation (batch_quantize, int8_quant.cpp:15-28,
// with the per-row scale of compute_minmax_scale).  inv_scale[r] = 1 / scale_r
// is the dequant multiplier (dequantize_from_int8 divides by scale, :38-44).
void oracle_quantize_rows(const float* x, int rows, int cols, int8_t* q, float* inv_scale) {
  for (int r = 0; r < rows; ++r) {
    const float scale = oracle_minmax_scale(x + (int64_t)r * cols, cols);
    oracle_quantize(x + (int64_t)r * cols, cols, scale, q + (int64_t)r * cols);
    inv_scale[r] = 1.0f / scale;
  }
}

// Per-output-column weight quantisation of W[K][N] (the INT8 weight format of
// this build; one scale per output channel, int8_quant.cpp semantics).
void oracle_quantize_cols(const float* w, int K, int N, int8_t* q, float* inv_scale) {
  std::vector<float> col(K);
  for (int n = 0; n < N; ++n) {
    for (int k = 0; k < K; ++k) col[k] = w[(int64_t)k * N + n];
    const float scale = oracle_minmax_scale(col.data(), K);
    for (int k = 0; k < K; ++k) {
      int32_t v = (int32_t)std::round(col[k] * scale);
      v = std::max(-128, std::min(127, v));
      q[(int64_t)k * N + n] = (int8_t)v;
    }
    inv_scale[n] = 1.0f / scale;
  }
}

// INT8 GEMM contract (attention_cpu/dnnl_matmul_int8.cpp:7-75):
//   acc[m,n] = sum_k int32(A[m,k]) * int32(W[k,n])            (exact)
//   y = float(acc) * (sa[m] * sw[n]) + bias[n]; act in {0 none, 1 relu, 2 gelu_erf}
// A: [M][K] row-major, W: [K][N] row-major (mlp.hpp:28-31 layout).
void oracle_i8_gemm(const int8_t* A, const int8_t* W, int32_t* acc_out, float* C, int M, int N,
                    int K, const float* sa, const float* sw, const float* bias, int act) {
#pragma omp parallel
  {
    std::vector<int32_t> acc(N);
#pragma omp for schedule(static)
    for (int m = 0; m < M; ++m) {
      std::fill(acc.begin(), acc.end(), 0);
      const int8_t* a = A + (int64_t)m * K;
      for (int k = 0; k < K; ++k) {
        const int32_t av = a[k];
        if (av == 0) continue;
        const int8_t* w = W + (int64_t)k * N;
        for (int n = 0; n < N; ++n) acc[n] += av * (int32_t)w[n];
      }
      if (acc_out) std::memcpy(acc_out + (int64_t)m * N, acc.data(), sizeof(int32_t) * N);
      if (C) {
        const float sam = sa ? sa[m] : 1.0f;
        for (int n = 0; n < N; ++n) {
          const float s = sam * (sw ? sw[n] : 1.0f);
          float y = (float)acc[n] * s;
          if (bias) y = y + bias[n];
          if (act == 1) y = std::max(0.0f, y);
          else if (act == 2) y = 0.5f * y * (1.0f + std::erf(y * 0.70710678118654752f));
          C[(int64_t)m * N + n] = y;
        }
      }
    }
  }
}

// LayerNorm<T>::forward restated (decoder/layer_norm.hpp:20-37), T = float:
// sequential mean, biased variance, inv_std = 1.0 / sqrt(var + eps) (double
// division of the float sqrt, as written), out = (x-mean)*inv_std*g + b.
// Test-only control (oracle_set_reduction_order): 1 sums the LayerNorm mean /
// variance and the decoder's attention dot products in REVERSE index order --
// the same maths with other fp32 roundings, the kind of difference a parallel
// reduction makes.  0 (default) is the reference's order; every pinned
// fixture and every parity test runs at 0.  tests/test_generate_free_run*.py use
// 1 to measure how far the INT8 decoder drifts from ITSELF free running when
// only the summation order changes (int8 rounding flips propagating through
// the KV cache): the yardstick for the GPU's free-running drift.
static int g_reverse_order = 0;

void oracle_layer_norm(const float* x, int rows, int cols, const float* gamma, const float* beta,
                       float eps, float* out) {
  const bool rev = g_reverse_order != 0;
  for (int r = 0; r < rows; ++r) {
    const float* in = x + (int64_t)r * cols;
    float* o = out + (int64_t)r * cols;
    float mean = 0;
    for (int i = 0; i < cols; ++i) mean += in[rev ? cols - 1 - i : i];
    mean /= cols;
    float var = 0;
    for (int i = 0; i < cols; ++i) {
      const int j = rev ? cols - 1 - i : i;
      var += (in[j] - mean) * (in[j] - mean);
    }
    var /= cols;
    const float inv_std = (float)(1.0 / std::sqrt(var + eps));
    for (int j = 0; j < cols; ++j) o[j] = (in[j] - mean) * inv_std * gamma[j] + beta[j];
  }
}

// MLP<float>::forward restated (decoder/mlp.hpp:23-41): fc1 [hid][inter]
// row-major + bias, ReLU, fc2 [inter][hid] + bias, float accumulation in
// index order starting from the bias.
void oracle_mlp_f32(const float* x, int rows, int hid, int inter, const float* w1, const float* b1,
                    const float* w2, const float* b2, float* out) {
  std::vector<float> h(inter);
  for (int b = 0; b < rows; ++b) {
    for (int i = 0; i < inter; ++i) {
      float sum = b1[i];
      for (int j = 0; j < hid; ++j) sum += x[(int64_t)b * hid + j] * w1[(int64_t)j * inter + i];
      h[i] = std::max(0.0f, sum);
    }
    for (int i = 0; i < hid; ++i) {
      float sum = b2[i];
      for (int j = 0; j < inter; ++j) sum += h[j] * w2[(int64_t)j * hid + i];
      out[(int64_t)b * hid + i] = sum;
    }
  }
}

// sample_from_logits (decoder/cuda_decoder.cu:7-14): argmax of logits/temperature,
// first maximum wins (std::max_element).
void oracle_argmax_rows(const float* logits, int rows, int V, int32_t* out) {
  for (int r = 0; r < rows; ++r) {
    const float* l = logits + (int64_t)r * V;
    out[r] = (int32_t)(std::max_element(l, l + V) - l);
  }
}

// ---------------------------------------------------------------------------
// Restated INT8Decoder decode step (reference order of
// decoder/decoder_block.hpp:41-62 plus the BUILD DECISION projections):
//   x = E[id]
//   per layer: a = LN1(x); qkv = i8gemm(quant(a), Wqkv); append k,v (fp16);
//              o = attn(q) over positions [0, pos]; x = i8gemm(quant(o), Wo);
//              a2 = LN2(x); h = relu(i8gemm(quant(a2), W1) + b1);
//              x = i8gemm(quant(h), W2) + b2
//   logits = x . E^T (fp16 E, double accumulation); next = argmax.
// The KV cache is contiguous per (layer, row, head) here (no paging): the
// paging itself is pinned separately by oracle_paged_attention.
// ---------------------------------------------------------------------------
struct oracle_model {
  int L, H, D, hid, inter, V, max_seq;
  const uint16_t* emb;                 // [V][hid] fp16 bits
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;  // [L][hid]
  const int8_t* wqkv; const float* sw_qkv;     // [L][hid][3hid], [L][3hid]
  const int8_t* wo;   const float* sw_o;       // [L][hid][hid],  [L][hid]
  const int8_t* w1;   const float* sw1; const float* b1;  // [L][hid][inter], [L][inter] x2
  const int8_t* w2;   const float* sw2; const float* b2;  // [L][inter][hid], [L][hid] x2
  // CUDADecoder (fp16 weights, decoder/cuda_decoder.cu): when hwqkv is set the
  // four projections use these fp16 [L][K][N] matrices instead of the int8
  // ones (sw_* unused): y = f16(x) . W in fp32 (+ bias, ReLU for fc1), with
  // the GEMM inputs rounded to fp16 as the GPU's f16 MFMA consumes them
  const uint16_t *hwqkv, *hwo, *hw1, *hw2;
};

// fp16-weight projection of the CUDADecoder restatement: out[m][n] =
// sum_k f16(x[m][k]) * W[k][n] in fp32 (k order), + bias[n], ReLU if act.
static void f16_gemm(const float* x, int M, int K, const uint16_t* W, int N, const float* bias,
                     int act, float* out) {
#pragma omp parallel
  {
    std::vector<float> xr(K);
#pragma omp for schedule(static)
    for (int m = 0; m < M; ++m) {
      for (int k = 0; k < K; ++k) xr[k] = half_to_float(float_to_half(x[(size_t)m * K + k]));
      float* o = out + (size_t)m * N;
      for (int n = 0; n < N; ++n) o[n] = 0.0f;
      for (int k = 0; k < K; ++k) {
        const float xv = xr[k];
        const uint16_t* wr = W + (size_t)k * N;
        for (int n = 0; n < N; ++n) o[n] += xv * half_to_float(wr[n]);
      }
      for (int n = 0; n < N; ++n) {
        float y = o[n] + (bias ? bias[n] : 0.0f);
        o[n] = act == 1 ? std::max(y, 0.0f) : y;
      }
    }
  }
}

struct OracleDecoder {
  oracle_model m;
  int B;
  std::vector<uint16_t> k, v;  // [L][B][H][max_seq][D] fp16 bits
  int64_t kv_index(int l, int b, int h, int t) const {
    return ((((int64_t)l * B + b) * m.H + h) * m.max_seq + t) * m.D;
  }
};

void* oracle_decoder_create(const oracle_model* model, int B) {
  auto* d = new OracleDecoder();
  d->m = *model;
  d->B = B;
  const size_t n = (size_t)model->L * B * model->H * model->max_seq * model->D;
  d->k.assign(n, 0);
  d->v.assign(n, 0);
  return d;
}

void oracle_decoder_destroy(void* h) { delete static_cast<OracleDecoder*>(h); }

uint16_t* oracle_decoder_kv_ptr(void* h, int layer, int which) {
  auto* d = static_cast<OracleDecoder*>(h);
  return (which == 0 ? d->k.data() : d->v.data()) + d->kv_index(layer, 0, 0, 0);
}

// One decode step for all B rows.  tokens[b] is the token at position pos[b];
// attention covers positions [0, pos[b]].  Runs the first `layers_to_run`
// layers (all if < 0) and the LM head + argmax if do_lm_head.
//
// Teacher forcing (oracle_decoder_step_forced): at each of a layer's four int8
// GEMM inputs (stage 0: LN1 output, 1: attention output, 2: LN2 output, 3: fc1
// output) the oracle quantises its own fp32 values as usual, compares them with
// the given activations (forced_q [L][4][B][Kmax] int8, forced_s [L][4][B] fp32
// scales, Kmax = max(hid, inter)), then continues from the GIVEN ones.  A fp32
// reduction-order difference can move a value across an int8 rounding boundary
// (one LSB); forcing keeps such a flip from propagating, so the rest of the
// step is compared at full precision.  stats [L][4][3]: number of int8 values
// that differ, their max |difference|, max rel. difference of the scales.
// attn_out (optional, [L][B][hid] fp32): every layer's attention output before
// the o_proj input conversion (int8 quantisation or the fp16 rounding of the
// CUDADecoder), for checks of the GPU's merged attention rows.
// forced_kv (optional, fp16 bits [L][B][2][H][D]): the K and V the step
// appends at pos, taken instead of the oracle's own fp16 rounding of its
// projection (the fp16 decoder's GEMM accumulates in another fp32 order, so a
// value can round one ulp apart); kv_stats [L][2]: values that differed, max
// |difference| / (one fp16 ulp + 1e-6 of the head's largest value).
static int decoder_step(void* handle, const int32_t* tokens, const int32_t* pos, float attn_scale,
                        int layers_to_run, int do_lm_head, float* x_out, float* logits_out,
                        int32_t* next_out, const int8_t* forced_q, const float* forced_s,
                        float* stats, float* attn_out, const uint16_t* forced_kv = nullptr,
                        float* kv_stats = nullptr);

int oracle_decoder_step(void* handle, const int32_t* tokens, const int32_t* pos, float attn_scale,
                        int layers_to_run, int do_lm_head, float* x_out, float* logits_out,
                        int32_t* next_out) {
  return decoder_step(handle, tokens, pos, attn_scale, layers_to_run, do_lm_head, x_out,
                      logits_out, next_out, nullptr, nullptr, nullptr, nullptr);
}

int oracle_decoder_step_forced(void* handle, const int32_t* tokens, const int32_t* pos,
                               float attn_scale, float* logits_out, int32_t* next_out,
                               const int8_t* forced_q, const float* forced_s, float* stats) {
  return decoder_step(handle, tokens, pos, attn_scale, -1, 1, nullptr, logits_out, next_out,
                      forced_q, forced_s, stats, nullptr);
}

// oracle_decoder_step / _step_forced with the per-layer attention outputs
// (forced_q NULL: a free step).  The fp16 CUDADecoder restatement is forced at
// its four fp16 GEMM inputs instead: forced_q then points to fp16 bits
// [L][4][B][Kmax] (uint16), forced_s is unused, and stats hold per (layer,
// stage): the fp16 values that differ from the oracle's own rounding, the max
// of |difference| / (one fp16 ulp of the value + 1e-6 of the row's largest
// value) -- <= 1 is a rounding flip --, and the max |difference| / row max.
int oracle_decoder_step_attn(void* handle, const int32_t* tokens, const int32_t* pos,
                             float attn_scale, float* logits_out, int32_t* next_out,
                             const int8_t* forced_q, const float* forced_s, float* stats,
                             float* attn_out, const uint16_t* forced_kv, float* kv_stats) {
  return decoder_step(handle, tokens, pos, attn_scale, -1, 1, nullptr, logits_out, next_out,
                      forced_q, forced_s, stats, attn_out, forced_kv, kv_stats);
}

static int decoder_step(void* handle, const int32_t* tokens, const int32_t* pos, float attn_scale,
                        int layers_to_run, int do_lm_head, float* x_out, float* logits_out,
                        int32_t* next_out, const int8_t* forced_q, const float* forced_s,
                        float* stats, float* attn_out, const uint16_t* forced_kv,
                        float* kv_stats) {
  auto* d = static_cast<OracleDecoder*>(handle);
  const oracle_model& m = d->m;
  const int B = d->B, H = m.H, D = m.D, hid = m.hid, inter = m.inter;
  for (int b = 0; b < B; ++b)
    if (pos[b] < 0 || pos[b] >= m.max_seq || tokens[b] < 0 || tokens[b] >= m.V) return 2;
  const int Lrun = layers_to_run < 0 ? m.L : std::min(layers_to_run, m.L);
  const bool f16w = m.hwqkv != nullptr;
  std::vector<float> x((size_t)B * hid), a((size_t)B * hid), qkv((size_t)B * 3 * hid),
      o((size_t)B * hid), h1((size_t)B * inter);
  std::vector<int8_t> qa((size_t)B * std::max(hid, inter));
  std::vector<float> sa(B);
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < hid; ++j) x[(size_t)b * hid + j] = half_to_float(m.emb[(size_t)tokens[b] * hid + j]);

  const int Kmax = std::max(hid, inter);
  // quantise `in` [B][K] into qa / sa, then (teacher forcing) compare with and
  // take the given activations of (layer, stage)
  auto quant = [&](int l, int stage, const float* in, int K) {
    oracle_quantize_rows(in, B, K, qa.data(), sa.data());
    if (!forced_q) return;
    const size_t slot = (size_t)l * 4 + stage;
    float n_diff = 0, max_diff = 0, max_srel = 0;
    for (int b = 0; b < B; ++b) {
      const int8_t* fq = forced_q + (slot * B + b) * Kmax;
      for (int j = 0; j < K; ++j) {
        const int dq = std::abs((int)qa[(size_t)b * K + j] - (int)fq[j]);
        if (dq) { n_diff += 1; max_diff = std::max(max_diff, (float)dq); }
        qa[(size_t)b * K + j] = fq[j];
      }
      const float fs = forced_s[slot * B + b];
      max_srel = std::max(max_srel, std::abs(fs - sa[b]) / std::max(std::abs(sa[b]), 1e-30f));
      sa[b] = fs;
    }
    if (stats) {
      stats[slot * 3 + 0] = n_diff;
      stats[slot * 3 + 1] = max_diff;
      stats[slot * 3 + 2] = max_srel;
    }
  };
  // fp16 decoder: round `in` [B][K] to fp16 as the GEMM consumes it, then
  // (teacher forcing) compare with and take the given fp16 activations
  auto force16 = [&](int l, int stage, float* in, int K) {
    if (!forced_q) return;
    const uint16_t* fh = reinterpret_cast<const uint16_t*>(forced_q);
    const size_t slot = (size_t)l * 4 + stage;
    float n_diff = 0, max_ratio = 0, max_abs = 0;
    for (int b = 0; b < B; ++b) {
      const uint16_t* f = fh + (slot * B + b) * Kmax;
      float* row = in + (size_t)b * K;
      float rmax = 0.f;
      for (int j = 0; j < K; ++j) rmax = std::max(rmax, std::fabs(row[j]));
      for (int j = 0; j < K; ++j) {
        const uint16_t own = float_to_half(row[j]);
        if (own != f[j]) {
          n_diff += 1;
          // one fp16 ulp (2^-10 relative) of the value, or 1e-6 of the row's
          // largest value for values near zero (subnormal ulps are tiny)
          const float d = std::fabs(half_to_float(own) - half_to_float(f[j]));
          const float tol = std::ldexp(std::fabs(half_to_float(own)), -10) + 1e-6f * rmax;
          max_ratio = std::max(max_ratio, d / std::max(tol, 1e-30f));
          max_abs = std::max(max_abs, d / std::max(rmax, 1e-30f));
        }
        row[j] = half_to_float(f[j]);
      }
    }
    if (stats) {
      stats[slot * 3 + 0] = n_diff;
      stats[slot * 3 + 1] = max_ratio;
      stats[slot * 3 + 2] = max_abs;
    }
  };
  for (int l = 0; l < Lrun; ++l) {
    const size_t lh = (size_t)l * hid;
    oracle_layer_norm(x.data(), B, hid, m.ln1_g + lh, m.ln1_b + lh, 1e-5f, a.data());
    if (f16w) {
      force16(l, 0, a.data(), hid);
      f16_gemm(a.data(), B, hid, m.hwqkv + (size_t)l * hid * 3 * hid, 3 * hid, nullptr, 0,
               qkv.data());
    } else {
      quant(l, 0, a.data(), hid);
      oracle_i8_gemm(qa.data(), m.wqkv + (size_t)l * hid * 3 * hid, nullptr, qkv.data(), B,
                     3 * hid, hid, sa.data(), m.sw_qkv + (size_t)l * 3 * hid, nullptr, 0);
    }
    // KV append (fp16 storage, round to nearest even), or the forced K / V
    float kv_nd = 0.f, kv_ratio = 0.f;
    for (int b = 0; b < B; ++b)
      for (int hh = 0; hh < H; ++hh)
        for (int which = 0; which < 2; ++which) {
          const float* src = qkv.data() + (size_t)b * 3 * hid + (1 + which) * hid + hh * D;
          uint16_t* dst = (which ? d->v.data() : d->k.data()) + d->kv_index(l, b, hh, pos[b]);
          const uint16_t* f =
              forced_kv ? forced_kv + ((((size_t)l * B + b) * 2 + which) * H + hh) * D : nullptr;
          float hmax = 0.f;
          if (f)
            for (int dd = 0; dd < D; ++dd) hmax = std::max(hmax, std::fabs(src[dd]));
          for (int dd = 0; dd < D; ++dd) {
            const uint16_t own = float_to_half(src[dd]);
            dst[dd] = own;
            if (!f || f[dd] == own) continue;
            kv_nd += 1.f;
            const float diff = std::fabs(half_to_float(own) - half_to_float(f[dd]));
            const float tol = std::ldexp(std::fabs(half_to_float(own)), -10) + 1e-6f * hmax;
            kv_ratio = std::max(kv_ratio, diff / std::max(tol, 1e-30f));
            dst[dd] = f[dd];
          }
        }
    if (kv_stats) {
      kv_stats[2 * l] = kv_nd;
      kv_stats[2 * l + 1] = kv_ratio;
    }
    // Attention: the reference scores are dot/temperature and its softmax divides
    // by temperature again (Appendix A #13); attn_scale = 1/temperature^2 folds
    // both.  exp(s - max) / (sum + 1e-6), out = sum p v.
#pragma omp parallel for collapse(2) schedule(dynamic)
    for (int b = 0; b < B; ++b) {
      for (int hh = 0; hh < H; ++hh) {
        const int Tb = pos[b] + 1;
        const float* qv = qkv.data() + (size_t)b * 3 * hid + hh * D;
        std::vector<float> sc(Tb), pr(Tb);
        const size_t base = d->kv_index(l, b, hh, 0);
        std::vector<float> kf(D);
        for (int t = 0; t < Tb; ++t) {
          const uint16_t* kr = d->k.data() + base + (size_t)t * D;
          float dot = 0.0f;
          for (int i = 0; i < D; ++i) {
            const int dd = g_reverse_order ? D - 1 - i : i;
            dot += qv[dd] * half_to_float(kr[dd]);
          }
          sc[t] = dot * attn_scale;
        }
        softmax_vec(sc.data(), Tb, 1.0f, pr.data());
        float* ov = o.data() + (size_t)b * hid + hh * D;
        for (int dd = 0; dd < D; ++dd) ov[dd] = 0.0f;
        for (int t = 0; t < Tb; ++t) {
          const uint16_t* vr = d->v.data() + base + (size_t)t * D;
          const float p = pr[t];
          for (int dd = 0; dd < D; ++dd) ov[dd] += p * half_to_float(vr[dd]);
        }
      }
    }
    if (attn_out) std::memcpy(attn_out + (size_t)l * B * hid, o.data(), sizeof(float) * B * hid);
    if (f16w) {
      force16(l, 1, o.data(), hid);
      f16_gemm(o.data(), B, hid, m.hwo + (size_t)l * hid * hid, hid, nullptr, 0, x.data());
      oracle_layer_norm(x.data(), B, hid, m.ln2_g + lh, m.ln2_b + lh, 1e-5f, a.data());
      force16(l, 2, a.data(), hid);
      f16_gemm(a.data(), B, hid, m.hw1 + (size_t)l * hid * inter, inter,
               m.b1 + (size_t)l * inter, 1, h1.data());
      force16(l, 3, h1.data(), inter);
      f16_gemm(h1.data(), B, inter, m.hw2 + (size_t)l * inter * hid, hid, m.b2 + lh, 0, x.data());
      continue;
    }
    quant(l, 1, o.data(), hid);
    oracle_i8_gemm(qa.data(), m.wo + (size_t)l * hid * hid, nullptr, x.data(), B, hid, hid,
                   sa.data(), m.sw_o + lh, nullptr, 0);
    oracle_layer_norm(x.data(), B, hid, m.ln2_g + lh, m.ln2_b + lh, 1e-5f, a.data());
    quant(l, 2, a.data(), hid);
    oracle_i8_gemm(qa.data(), m.w1 + (size_t)l * hid * inter, nullptr, h1.data(), B, inter, hid,
                   sa.data(), m.sw1 + (size_t)l * inter, m.b1 + (size_t)l * inter, 1);
    quant(l, 3, h1.data(), inter);
    oracle_i8_gemm(qa.data(), m.w2 + (size_t)l * inter * hid, nullptr, x.data(), B, hid, inter,
                   sa.data(), m.sw2 + lh, m.b2 + lh, 0);
  }
  if (x_out) std::memcpy(x_out, x.data(), sizeof(float) * x.size());
  if (!do_lm_head) return 0;
  std::vector<float> logits((size_t)B * m.V);
#pragma omp parallel for schedule(static)
  for (int vv = 0; vv < m.V; ++vv) {
    const uint16_t* e = m.emb + (size_t)vv * hid;
    for (int b = 0; b < B; ++b) {
      double acc = 0.0;
      const float* xb = x.data() + (size_t)b * hid;
      for (int j = 0; j < hid; ++j) acc += (double)xb[j] * (double)half_to_float(e[j]);
      logits[(size_t)b * m.V + vv] = (float)acc;
    }
  }
  if (logits_out) std::memcpy(logits_out, logits.data(), sizeof(float) * logits.size());
  if (next_out) oracle_argmax_rows(logits.data(), B, m.V, next_out);
  return 0;
}

void oracle_set_reduction_order(int reverse) { g_reverse_order = reverse ? 1 : 0; }
int oracle_get_reduction_order() { return g_reverse_order; }

int oracle_num_threads() { return omp_get_max_threads(); }
// The CPU baseline sets its thread count explicitly (OMP_NUM_THREADS is read
// once, when the OpenMP runtime starts, possibly before this library loads).
void oracle_set_num_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

}  // extern "C"
