// Decoder runtime (host side, compiled as HIP): CUDADecoder / INT8Decoder
// (decoder/cuda_decoder.{hpp,cu}, decoder/int8_decoder.{hpp,cpp}) re-designed
// for batched incremental decode on one MI355X.
//
// One decode step for all rows (reference layer order of
// DecoderBlock<T>::forward, decoder/decoder_block.hpp:41-62 — no residuals —
// plus the BUILD DECISION projections):
//   embed -> per layer { LN1+quant -> qkv GEMM -> KV append -> paged attention
//   -> quant -> o GEMM -> LN2+quant -> fc1 GEMM (+b1, ReLU) -> quant -> fc2 GEMM
//   (+b2) } -> LM head (tied fp16 embedding) -> argmax -> advance positions.
// The reference re-embeds and recomputes the whole prefix every step
// (decoder/cuda_decoder.cu:52-57) and runs B = 1; here the KV cache is
// appended in place and the step is O(T) per row.
//
// The device part of a step is captured once per batch size into a hipGraph
// and replayed; per-step state (positions, context lengths, tokens) lives in
// device memory, so replays need no re-capture.  Only page allocation (a new
// page every page_size tokens, copy-on-write of forked pages) happens on the
// host between replays and is pushed with kv_cache_sync().
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "common.hpp"
#include "gemm.hpp"
#include "kv_cache_impl.hpp"
#include "pa_decode.hpp"
#include "row_ops.hpp"

using namespace llm;

// f[1] = f[0], f[0] = 0 in one device atomic: the fused o_proj's range flag
// read and cleared (llm_decoder::report_range)
__global__ void take_flag_kernel(int* f) { f[1] = atomicExch(f, 0); }

namespace {

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  int alloc(size_t count) {
    if (p) { (void)hipFree(p); p = nullptr; }
    n = count;
    if (count == 0) return LLM_OK;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(LLM_ERR_OOM, "decoder: device allocation of " + std::to_string(count * sizeof(T)) +
                                   " bytes failed");
    }
    return LLM_OK;
  }
};

#define RET_IF(x) do { int _rc = (x); if (_rc) return _rc; } while (0)

}  // namespace

struct llm_decoder {
  llm_decoder_config cfg{};
  int L = 0, H = 0, D = 0, hid = 0, inter = 0, V = 0, TS = 0, max_tiles = 0, maxB = 0;
  int wdtype = LLM_I8;
  int pps = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;

  // weights
  DevBuf<uint16_t> emb;
  DevBuf<uint8_t> emb_packed;  // LM-head copy of emb in B-fragment order
  DevBuf<float> ln1_g, ln1_b, ln2_g, ln2_b, b1, b2, sw_qkv, sw_o, sw1, sw2;
  DevBuf<uint8_t> wqkv, wo, w1, w2;  // packed, L consecutive blocks
  // FP16: W_o again as per-head column slices for the fused o_proj,
  // [L][H][D/8][hid][8] (PaRowOutputs::wo_heads)
  DevBuf<uint16_t> wo_heads;
  size_t sz_qkv = 0, sz_o = 0, sz_1 = 0, sz_2 = 0;
  bool weights_ready = false;
  int w_keep = 0;  // the GEMM weights fit the Infinity Cache: keep them there (w_keep_for)

  // KV
  kv_cache* kv = nullptr;

  // activations / state
  DevBuf<float> x, qkv, o, h1, logits, sa;
  DevBuf<float> lm_pv;    // [max_batch][lm_nwg] LM-head argmax partials
  DevBuf<int32_t> lm_pi;
  int lm_nwg = 0;
  DevBuf<int8_t> qa;
  DevBuf<uint16_t> a16;
  // FP16: the fused o_proj's int64 columns [max_batch][hid] (zero between
  // attention launches: the adder completing a column clears it); oacc_run:
  // llm_decoder_run_attention's own set (allocated on first use), so a timed
  // run never mixes its arrivals with an in-flight step's; oflag: the range
  // guard's device flag of the steps (common.hpp oacc_term), h_oflag its pinned
  // host copy (written and read under mu only); oflag_run: run_attention's own
  // flag, so a clamp in a timing re-run is never blamed on a step.
  // range_clamped: a clamp was reported since the last begin / generate (what
  // llm_decoder_oproj_status returns; the device flag is cleared on report)
  DevBuf<long long> oacc, oacc_run;
  DevBuf<int> oflag, oflag_run;
  int* h_oflag = nullptr;
  int range_clamped = 0;
  // beam-group attention (row_group 4): the dynamic tile counters
  // (PaRowOutputs::beam_ctr), zero at create and left at zero by every launch
  DevBuf<unsigned> beam_ctr;
  int oproj_range_status();
  int report_range(int flag);
  DevBuf<int32_t> tokens, pos, ctx;
  DevBuf<uint8_t> attn_ws;
  size_t attn_ws_bytes = 0;

  int batch = 0;
  std::vector<int> h_pos;  // host mirror of the next position of each row

  hipGraphExec_t graph = nullptr;
  int graph_batch = -1;

  // activation taps (llm_decoder_set_taps): the int8 GEMM inputs and row scales
  // of every layer, copied out by the step for teacher-forced parity checks
  int8_t* tap_q = nullptr;
  float* tap_s = nullptr;
  int tap(int l, int stage, const struct Rows& R, int K, hipStream_t st);
  int layer_norm_into(WeightGemm& g, const struct Rows& R, const float* gamma, const float* beta,
                      hipStream_t st, float* zero_x = nullptr);
  LnSource embed_src;  // set by step_head: the next LayerNorm reads E[token] rows

  ~llm_decoder() {
    if (h_oflag) (void)hipHostFree(h_oflag);
    if (graph) (void)hipGraphExecDestroy(graph);
    if (kv) kv_cache_destroy(kv);
    if (stream) (void)hipStreamDestroy(stream);
  }

  int row_group = 1;  // beam width of llm_decoder_begin_beams (beam-aware attention)
  // sampling (llm_decoder_set_sampling); greedy argmax by default, as the
  // reference's sample_from_logits (decoder/cuda_decoder.cu:7-14)
  float temperature = 0.f;
  int top_k = 0;
  float top_p = 1.f;
  uint64_t sample_seed = 0;
  bool use_graph = true;  // LLM_GRAPH=0: eager launches (per-kernel profiling)
  int qa_ld = 0;
  size_t b16 = 0;  // max_batch rounded up to 16-row tiles

  int layer_pre(int l, hipStream_t st, const struct Rows& R);
  int layer_attn(int l, hipStream_t st, const struct Rows& R, PaPlan* plan = nullptr);
  bool quant_prologue(const struct Rows& R) const;
  bool oproj_fusable(const struct Rows& R);
  bool wgm_quant_ok(const struct Rows& R);
  bool fc2_split(const struct Rows& R) const;
  int layer_post(int l, hipStream_t st, const struct Rows& R);
  struct Rows step_rows(int r0, int n, uint8_t* ws);
  int step_head(hipStream_t st, int r0, int n);
  int step_tail(hipStream_t st, int r0, int n);
  int next_tokens(const float* xr, int n, int r0, const int32_t* ctr, hipStream_t st,
                  int32_t* adv_pos = nullptr, int32_t* adv_ctx = nullptr);
  int enqueue_step(hipStream_t st);
  int run_step(const int32_t* tokens_host, float* logits_dev, int32_t* next_host, hipStream_t st);

  // chunked prefill (llm_decoder_prefill): buffers for one chunk of tokens
  static constexpr int kPrefillChunk = 512;
  DevBuf<float> px, pq, po, ph1, psa;
  DevBuf<uint8_t> pact, pws;
  DevBuf<int32_t> pmeta;  // [4][chunk]: pos, ctx, page-table row, token
  size_t pws_bytes = 0;
  int pf_cap = 0;
  int prefill(int row, const int32_t* toks, int n, hipStream_t st);
};

static int check_cfg(const llm_decoder_config& c) {
  LLM_REQUIRE(c.num_layers > 0 && c.num_heads > 0 && c.head_dim > 0 && c.vocab_size > 0 &&
                  c.max_seq_len > 0,
              "decoder: num_layers/num_heads/head_dim/vocab_size/max_seq_len must be positive");
  LLM_REQUIRE(c.hidden_dim == c.num_heads * c.head_dim,
              "decoder: hidden_dim must equal num_heads * head_dim");
  LLM_REQUIRE(c.weight_dtype == LLM_I8 || c.weight_dtype == LLM_F16, "decoder: weight_dtype");
  return LLM_OK;
}

extern "C" int llm_decoder_create(const llm_decoder_config* cfg_in, llm_decoder** out) {
  LLM_REQUIRE(cfg_in && out, "llm_decoder_create: NULL");
  llm_decoder_config c = *cfg_in;
  if (c.inter_dim <= 0) c.inter_dim = 4 * c.hidden_dim;
  if (c.page_size <= 0) c.page_size = 16;
  if (c.max_batch <= 0) c.max_batch = 1;
  if (c.attn_scale == 0.f) c.attn_scale = 1.f;
  RET_IF(check_cfg(c));
  LLM_REQUIRE(c.hidden_dim % 64 == 0 && c.inter_dim % 64 == 0 && c.inter_dim <= 16384,
              "decoder: hidden_dim and inter_dim must be multiples of 64 (packed GEMM "
              "activations), inter_dim <= 16384");
  std::unique_ptr<llm_decoder> d(new llm_decoder());
  d->cfg = c;
  d->L = c.num_layers; d->H = c.num_heads; d->D = c.head_dim; d->hid = c.hidden_dim;
  d->inter = c.inter_dim; d->V = c.vocab_size; d->TS = c.page_size;
  d->max_tiles = (c.max_seq_len + c.page_size - 1) / c.page_size;
  d->maxB = c.max_batch;
  d->wdtype = c.weight_dtype;
  LLM_HIP_RET(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  long long pages = c.num_pages > 0 ? c.num_pages
                                     : (long long)d->maxB * d->L * d->H * d->max_tiles;
  RET_IF(kv_cache_create(d->L, d->maxB, d->H, d->D, d->TS, d->max_tiles, pages, &d->kv));
  const int B = d->maxB, hid = d->hid, inter = d->inter;
  RET_IF(d->x.alloc((size_t)B * hid));
  RET_IF(d->qkv.alloc((size_t)B * 3 * hid));
  RET_IF(d->o.alloc((size_t)B * hid));
  RET_IF(d->h1.alloc((size_t)B * inter));
  RET_IF(d->logits.alloc((size_t)B * d->V));
  d->lm_nwg = lm_head_workgroups(d->V);
  RET_IF(d->lm_pv.alloc((size_t)B * d->lm_nwg));
  RET_IF(d->lm_pi.alloc((size_t)B * d->lm_nwg));
  RET_IF(d->sa.alloc((size_t)B));
  const size_t B16 = ((size_t)B + 15) / 16 * 16;  // packed-A tiles are 16 rows
  RET_IF(d->qa.alloc(B16 * std::max(hid, inter)));
  if (d->wdtype == LLM_F16) {
    RET_IF(d->a16.alloc(2 * B16 * std::max(hid, inter)));  // act, act2
    RET_IF(d->oacc.alloc((size_t)B * hid));
    LLM_HIP_RET(hipMemset(d->oacc.p, 0, sizeof(long long) * B * hid));
    RET_IF(d->oflag.alloc(2));  // [0] the flag, [1] take_flag_kernel's result
    LLM_HIP_RET(hipMemset(d->oflag.p, 0, 2 * sizeof(int)));
    LLM_HIP_RET(hipHostMalloc(reinterpret_cast<void**>(&d->h_oflag), sizeof(int)));
    *d->h_oflag = 0;
  }
  RET_IF(d->beam_ctr.alloc(2 * (((size_t)B + 3) / 4) * d->H));
  LLM_HIP_RET(hipMemset(d->beam_ctr.p, 0, sizeof(unsigned) * d->beam_ctr.n));
  d->b16 = B16;
  RET_IF(d->tokens.alloc((size_t)B));
  RET_IF(d->pos.alloc((size_t)B));
  RET_IF(d->ctx.alloc((size_t)B));
  d->pps = 0;  // balanced splits derived on device from each row's context
  d->attn_ws_bytes = 16;
  for (int b = 1; b <= B; ++b)  // any batch size up to max_batch
    d->attn_ws_bytes = std::max(d->attn_ws_bytes,
                                pa_decode_workspace_bytes(b, d->H, d->D, d->max_tiles, 0));
  RET_IF(d->attn_ws.alloc(std::max<size_t>(d->attn_ws_bytes, 16)));
  d->qa_ld = std::max(hid, inter);
  // Splitting the rows into two micro-batches on two streams was measured and
  // removed: one graph with two branches, two graphs on two
  // streams, ping-pong attention and a CU partition all lose (C2 -11..-13 %,
  // C4 -5 %, C3 -0.5..+1 %: the branches do not overlap usefully, and a
  // saturating KV scan slows the other half's glue 4-8x).
  d->use_graph = env_int("LLM_GRAPH", 1) != 0;
  d->h_pos.assign(B, 0);
  *out = d.release();
  return LLM_OK;
}

extern "C" void llm_decoder_destroy(llm_decoder* d) {
  if (!d) return;
  if (d->stream) (void)hipStreamSynchronize(d->stream);
  delete d;
}

extern "C" kv_cache* llm_decoder_kv(llm_decoder* d) { return d ? d->kv : nullptr; }

// ---------------------------------------------------------------------------
// weights
// ---------------------------------------------------------------------------
template <typename T>
static int upload(DevBuf<T>& dst, const T* src, size_t n, const char* what) {
  LLM_REQUIRE(src != nullptr, std::string("decoder weights: ") + what + " is NULL");
  RET_IF(dst.alloc(n));
  LLM_HIP_RET(hipMemcpy(dst.p, src, n * sizeof(T), hipMemcpyHostToDevice));
  return LLM_OK;
}

// Upload L row-major [K][N] matrices and pack each into MFMA fragment order.
static int upload_packed(DevBuf<uint8_t>& dst, size_t& per_layer, const void* src, int L, int K,
                         int N, int dtype, const char* what) {
  LLM_REQUIRE(src != nullptr, std::string("decoder weights: ") + what + " is NULL");
  const size_t esz = dtype == LLM_I8 ? 1 : 2;
  per_layer = gemm_packed_bytes(dtype, K, N);
  RET_IF(dst.alloc(per_layer * L));
  void* tmp = nullptr;
  LLM_HIP_RET(hipMalloc(&tmp, (size_t)K * N * esz));
  int rc = LLM_OK;
  for (int l = 0; l < L && rc == LLM_OK; ++l) {
    const char* s = static_cast<const char*>(src) + (size_t)l * K * N * esz;
    if (hipMemcpy(tmp, s, (size_t)K * N * esz, hipMemcpyHostToDevice) != hipSuccess) {
      rc = fail(LLM_ERR_HIP, "decoder weights: upload failed");
      break;
    }
    rc = gemm_pack_weights(dtype, tmp, dst.p + per_layer * l, K, N, nullptr);
  }
  (void)hipDeviceSynchronize();
  (void)hipFree(tmp);
  return rc;
}

static int upload_common(llm_decoder* d, const uint16_t* emb, const float* ln1_g,
                         const float* ln1_b, const float* ln2_g, const float* ln2_b) {
  const size_t Lh = (size_t)d->L * d->hid;
  RET_IF(upload(d->emb, emb, (size_t)d->V * d->hid, "emb"));
  RET_IF(d->emb_packed.alloc(lm_head_packed_bytes(d->V, d->hid)));
  LLM_HIP_RET(launch_lm_pack(d->emb.p, d->emb_packed.p, d->V, d->hid, nullptr));
  LLM_HIP_RET(hipDeviceSynchronize());
  RET_IF(upload(d->ln1_g, ln1_g, Lh, "ln1_g"));
  RET_IF(upload(d->ln1_b, ln1_b, Lh, "ln1_b"));
  RET_IF(upload(d->ln2_g, ln2_g, Lh, "ln2_g"));
  RET_IF(upload(d->ln2_b, ln2_b, Lh, "ln2_b"));
  return LLM_OK;
}

// The weight GEMMs load with the default cache policy (lines stay in the
// 256 MiB Infinity Cache, so the next step's GEMMs hit there) when the whole
// weight set fits well inside it; the KV stream is loaded non-temporal and
// does not displace them.  Larger models stream their weights nt (read once
// per step: keeping them would only churn the cache).  Same-box A/B, two
// runs each (profiles/r03/wkeep_ab.txt): C2 (170 MB of weights) +1.7 / +2.1 %
// kept; C4 (1.2 GB) -2.3 / -2.6 % kept, so nt there.
static int w_keep_for(const llm_decoder* d) {
  const size_t bytes = (d->sz_qkv + d->sz_o + d->sz_1 + d->sz_2) * (size_t)d->L;
  return bytes <= (size_t)192 << 20;
}

extern "C" int llm_decoder_set_int8_weights(llm_decoder* d, const llm_int8_weights* w) {
  LLM_REQUIRE(d && w, "llm_decoder_set_int8_weights: NULL");
  LLM_REQUIRE(d->wdtype == LLM_I8, "llm_decoder_set_int8_weights: decoder is not INT8");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  const int L = d->L, hid = d->hid, inter = d->inter;
  RET_IF(upload_common(d, w->emb, w->ln1_g, w->ln1_b, w->ln2_g, w->ln2_b));
  RET_IF(upload_packed(d->wqkv, d->sz_qkv, w->wqkv, L, hid, 3 * hid, LLM_I8, "wqkv"));
  RET_IF(upload_packed(d->wo, d->sz_o, w->wo, L, hid, hid, LLM_I8, "wo"));
  RET_IF(upload_packed(d->w1, d->sz_1, w->w1, L, hid, inter, LLM_I8, "w1"));
  RET_IF(upload_packed(d->w2, d->sz_2, w->w2, L, inter, hid, LLM_I8, "w2"));
  RET_IF(upload(d->sw_qkv, w->sw_qkv, (size_t)L * 3 * hid, "sw_qkv"));
  RET_IF(upload(d->sw_o, w->sw_o, (size_t)L * hid, "sw_o"));
  RET_IF(upload(d->sw1, w->sw1, (size_t)L * inter, "sw1"));
  RET_IF(upload(d->sw2, w->sw2, (size_t)L * hid, "sw2"));
  RET_IF(upload(d->b1, w->b1, (size_t)L * inter, "b1"));
  RET_IF(upload(d->b2, w->b2, (size_t)L * hid, "b2"));
  d->w_keep = w_keep_for(d);
  d->graph_batch = -1;
  d->weights_ready = true;
  return LLM_OK;
}

extern "C" int llm_decoder_set_f16_weights(llm_decoder* d, const llm_f16_weights* w) {
  LLM_REQUIRE(d && w, "llm_decoder_set_f16_weights: NULL");
  LLM_REQUIRE(d->wdtype == LLM_F16, "llm_decoder_set_f16_weights: decoder is not FP16");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  const int L = d->L, hid = d->hid, inter = d->inter;
  RET_IF(upload_common(d, w->emb, w->ln1_g, w->ln1_b, w->ln2_g, w->ln2_b));
  RET_IF(upload_packed(d->wqkv, d->sz_qkv, w->wqkv, L, hid, 3 * hid, LLM_F16, "wqkv"));
  RET_IF(upload_packed(d->wo, d->sz_o, w->wo, L, hid, hid, LLM_F16, "wo"));
  // the fused o_proj's head slices: [h][kg][n][j] = W_o[h D + 8 kg + j][n] (a
  // second copy of W_o, L * hid^2 fp16), only where the fused o_proj can run
  // (oproj_fusable); the step then reads these instead of the packed W_o, so
  // the bytes a step streams (w_keep_for) are unchanged
  d->wo_heads.alloc(0);
  if (d->D % 8 == 0 && d->D <= 128 && d->H <= 64 && oproj_fuse_on()) {
    const int D = d->D, KG = D / 8;
    const uint16_t* src = static_cast<const uint16_t*>(w->wo);
    std::vector<uint16_t> sl((size_t)hid * hid);
    RET_IF(d->wo_heads.alloc((size_t)L * hid * hid));
    for (int l = 0; l < L; ++l) {
      const uint16_t* wl = src + (size_t)l * hid * hid;
      for (int h = 0; h < d->H; ++h)
        for (int kg = 0; kg < KG; ++kg)
          for (int n = 0; n < hid; ++n)
            for (int j = 0; j < 8; ++j)
              sl[(((size_t)h * KG + kg) * hid + n) * 8 + j] = wl[(size_t)(h * D + 8 * kg + j) * hid + n];
      LLM_HIP_RET(hipMemcpy(d->wo_heads.p + (size_t)l * hid * hid, sl.data(),
                            sizeof(uint16_t) * hid * hid, hipMemcpyHostToDevice));
    }
  }
  RET_IF(upload_packed(d->w1, d->sz_1, w->w1, L, hid, inter, LLM_F16, "w1"));
  RET_IF(upload_packed(d->w2, d->sz_2, w->w2, L, inter, hid, LLM_F16, "w2"));
  RET_IF(upload(d->b1, w->b1, (size_t)L * inter, "b1"));
  RET_IF(upload(d->b2, w->b2, (size_t)L * hid, "b2"));
  d->w_keep = w_keep_for(d);
  d->graph_batch = -1;
  d->weights_ready = true;
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// step
// ---------------------------------------------------------------------------
// The rows one layer pass works on: the decode rows (rows r0.. of the step
// buffers, one token each) or a prefill chunk (n tokens of one sequence,
// beam_rows[m] = its page-table row).  Every buffer is row-indexed.
struct Rows {
  int n = 0;
  float* x = nullptr;   // [n][hid] residual-free hidden state
  float* q = nullptr;   // [n][hid] q of the fused qkv projection
  float* o = nullptr;   // [n][hid] attention output (fp32)
  float* h1 = nullptr;  // [n][inter]
  void* act = nullptr;  // packed-A GEMM input (int8 or fp16), 16-row tiles
  void* act2 = nullptr; // fp16 decoder: fc2's packed input (written by fc1 while act is read)
  float* sa = nullptr;  // [n] int8 row scales
  const int32_t* pos = nullptr;  // [n] position written this pass
  const int32_t* ctx = nullptr;  // [n] context length attended (pos + 1)
  const int32_t* beam_rows = nullptr;  // page-table row per row; NULL: table_row0 + m
  int table_row0 = 0;
  int row_group = 1;
  // INT8 rows too wide for the o_proj quantising prologue (wgm_quant_ok): the
  // attention writes fp32 rows merged in the workgroup and a quantise launch
  // follows it
  bool wgm_quant = false;
  // prefill chunk (row >= 0): the n rows are positions p0 .. p0+n-1 of page-table
  // row prefill_row, attended causally by the MFMA prefill kernel
  int prefill_row = -1;
  int prefill_p0 = 0;
  uint8_t* attn_ws = nullptr;
  size_t attn_ws_bytes = 0;
  // FP16 decode rows: the o_proj runs inside the attention's workgroup merge
  // (oproj_fusable) through these int64 columns and writes oproj_out (x, or a
  // scratch row for llm_decoder_run_attention); no o_proj launch
  long long* oacc = nullptr;
  float* oproj_out = nullptr;
  int* oflag = nullptr;  // the range guard's flag for these columns
};

// Activations feeding a weight GEMM (qa int8 / a16 fp16) are kept in packed-A
// order (common.hpp a_frag_off_*): their producers (LayerNorm+quant, the
// attention merge, the row quantiser) write MFMA A-fragments directly, so
// every GEMM A load is one coalesced 1 KiB read.  Row offsets r0 are
// multiples of 16, so r0 is the same base offset in both layouts (r0 * K
// elements).
int llm_decoder::layer_pre(int l, hipStream_t st, const Rows& R) {
  const size_t lh = (size_t)l * hid;
  pa_kv_view view;
  RET_IF(kv_cache_view(kv, l, &view));
  KvAppendView app;
  app.pos = R.pos;
  app.page_table = view.page_table + (size_t)R.table_row0 * H * view.max_tiles;
  app.rows = R.beam_rows;
  app.k_pool = kv_cache_k_pool(kv);
  app.v_pool = kv_cache_v_pool(kv);
  app.num_beams = view.num_beams - R.table_row0;
  app.max_tiles = view.max_tiles;
  app.page_size = TS;
  app.num_pages = view.num_pages;
  app.H = H;
  app.D = D;
  app.page_stride = (size_t)view.page_stride / sizeof(_Float16);
  WeightGemm g;
  g.dtype = wdtype;
  g.a_packed = 1;
  g.w_keep = w_keep;
  g.A = R.act;
  g.W_packed = wqkv.p + sz_qkv * l;
  g.M = R.n; g.N = 3 * hid; g.K = hid;
  g.C = R.q; g.c_cols = hid; g.c_ld = hid;  // q only: K and V go straight into the pages
  g.kv = &app;
  if (wdtype == LLM_I8) g.sa = R.sa, g.sw = sw_qkv.p + (size_t)l * 3 * hid;
  RET_IF(layer_norm_into(g, R, ln1_g.p + lh, ln1_b.p + lh, st));
  RET_IF(weight_gemm(g, st));
  return tap(l, 0, R, hid, st);
}

// LN(x) as the GEMM's A: fused into the GEMM as its LayerNorm prologue when
// the rows' A image fits in LDS (decode rows), else a LayerNorm (+ quant)
// launch writing the packed A the GEMM reads.
int llm_decoder::layer_norm_into(WeightGemm& g, const Rows& R, const float* gamma,
                                 const float* beta, hipStream_t st, float* zero_x) {
  // the step's first LayerNorm reads the token embedding rows (step_head)
  LnSource src = embed_src;
  embed_src = LnSource{};
  src.zero_x = zero_x;  // (the LayerNorm launch only: the caller checks fc2_split)
  if (R.prefill_row < 0 && ln_fusable(wdtype, R.n, hid)) {
    g.ln_x = R.x; g.ln_g = gamma; g.ln_b = beta; g.ln_eps = 1e-5f;
    g.ln_emb = src.emb; g.ln_tok = src.tok; g.ln_V = src.V;
    if (tap_q) { g.act_out = R.act; g.sa_out = R.sa; }  // the taps read A and the scales back
    return LLM_OK;
  }
  const LnSource* pp = src.emb || src.zero_x ? &src : nullptr;
  if (wdtype == LLM_I8)
    LLM_HIP_RET(launch_layernorm_quant(R.x, R.n, hid, gamma, beta, 1e-5f, nullptr,
                                       static_cast<int8_t*>(R.act), R.sa, st, 1, pp));
  else
    LLM_HIP_RET(launch_layernorm_f16(R.x, R.n, hid, gamma, beta, 1e-5f, R.act, st, 1, pp));
  return LLM_OK;
}

// INT8 decode rows whose o_proj can quantise its own input (gemm.hip
// quant_prologue_ok): the attention writes fp32 rows, merging its splits in
// the workgroup, and the o_proj prologue quantises them per row -- no merge
// launch.  Beam groups keep the merge launch (the beam kernel's workgroups
// are 4 beams of one split), as do prefill chunks.
bool llm_decoder::quant_prologue(const Rows& R) const {
  return wdtype == LLM_I8 && R.prefill_row < 0 && R.row_group == 1 &&
         quant_prologue_ok(R.n, hid, hid);
}

// FP16 decode rows whose o_proj the attention's workgroup merge can run
// (pa_decode.hip, OPROJ): each (row, head) workgroup multiplies its merged
// head by W_o's rows for that head and adds the products into the int64
// columns R.oacc; the adder completing a column writes x (what the o_proj
// GEMM wrote).  One launch per layer fewer (C2: the 4.9 us o_proj GEMM).
// Needs the workgroup-merge form (2..8 splits), head_dim <= 128 and <= 64
// heads; otherwise the o_proj GEMM runs as before.
bool llm_decoder::oproj_fusable(const Rows& R) {
  if (wdtype != LLM_F16 || R.prefill_row >= 0 || R.row_group != 1 || R.beam_rows || !wo_heads.p ||
      D > 128 || H > 64 || !oproj_fuse_on())
    return false;
  Rows r = R;
  r.oacc = oacc.p;
  r.oproj_out = R.x;
  r.oflag = oflag.p;
  PaPlan p;
  if (layer_attn(0, stream, r, &p) != LLM_OK) return false;
  return (p.form & LLM_PA_FORM_OPROJ) != 0;
}

// INT8 decode rows whose o_proj cannot quantise its own input (hidden >
// 2048: C5's 4096, 256 KB of fp32 rows per 16-row workgroup): when the plan
// with fp32 rows is the workgroup merge (<= 8 splits), the attention merges
// its splits in the workgroup and one quantise launch writes the packed int8
// o_proj input -- in place of split + pa_merge_row_kernel (C5: 5 splits of
// 103 pages -> 8 of 65 merged in the workgroup).
bool llm_decoder::wgm_quant_ok(const Rows& R) {
  if (wdtype != LLM_I8 || R.prefill_row >= 0 || R.row_group != 1 || R.beam_rows ||
      quant_prologue(R))
    return false;
  Rows r = R;
  r.wgm_quant = true;
  PaPlan p;
  if (layer_attn(0, stream, r, &p) != LLM_OK) return false;
  return (p.form & 15) == LLM_PA_FORM_WG_MERGE;
}

// INT8 decode rows <= 16 (the 4- and 8-GPU points of C3's strong curve): fc2's
// 128 column tiles leave half the CUs idle, so it runs as two k slices that
// each add their dequantised half into x (fp32 atomics; two addends commute,
// so x is the same bits whichever lands first).  x must be zero when fc2
// starts: the LN2 launch, the last reader of the o_proj output in x, writes
// zeros over the rows after loading them.  Standalone (scripts/tune_gemm_sk.py,
// profiles/r05/gemm_small_m.txt): fc2 at M = 8 6.86 -> 5.67 us, M = 16 7.53 ->
// 5.95 us.
// Round 6: also at 33..64 rows when inter >= 16384 (C5's fc2, K 16384): every
// workgroup of the one-slice form reads all of A, 1 MB, the k slices half of
// it (gemm_impl.hpp narrow_decode_tile).
bool llm_decoder::fc2_split(const Rows& R) const {
  return wdtype == LLM_I8 && R.prefill_row < 0 &&
         (R.n <= 16 || (R.n > 32 && R.n <= 64 && inter >= 16384)) &&
         !ln_fusable(wdtype, R.n, hid) && inter / 64 >= 16;
}

int llm_decoder::layer_attn(int l, hipStream_t st, const Rows& R, PaPlan* plan) {
  pa_kv_view view;
  RET_IF(kv_cache_view(kv, l, &view));
  view.page_table += (size_t)R.table_row0 * H * view.max_tiles;  // rows r0..
  view.num_beams -= R.table_row0;
  if (R.prefill_row >= 0 && pa_prefill_supported(&view) && !plan) {
    // one MFMA pass over the chunk (K/V pages read once per 32 queries), then
    // the o_proj input conversion the decode merge would have fused
    PaRowOutputs ro;
    ro.pack = 1;
    ro.keep_out = 0;
    if (wdtype == LLM_I8) {
      ro.q = static_cast<int8_t*>(R.act);
      ro.inv_scale = R.sa;
    } else {
      ro.out16 = R.act;
    }
    return pa_prefill_internal(&view, R.q, hid, R.o, hid, R.prefill_row, R.prefill_p0, R.n,
                               cfg.attn_scale, R.attn_ws, R.attn_ws_bytes, st, &ro);
  }
  // the split merge also produces the o_proj input (packed int8 + scale, or fp16);
  // the fp32 rows are only needed by a single-split (direct) launch
  PaRowOutputs ro;
  ro.pack = 1;
  ro.keep_out = 0;
  if (quant_prologue(R) || R.wgm_quant) {
    ro.f32_rows = 1;  // fp32 rows in R.o, quantised by the o_proj prologue or the launch below
  } else if (wdtype == LLM_I8) {
    ro.q = static_cast<int8_t*>(R.act);
    ro.inv_scale = R.sa;
  } else if (R.oacc) {
    ro.o_acc = R.oacc;
    ro.o_x = R.oproj_out;
    ro.wo_heads = wo_heads.p + (size_t)l * hid * hid;
    ro.o_n = hid;
    ro.o_flag = R.oflag;
    ro.out16 = tap_q ? R.act : nullptr;  // the taps read the packed o_proj input
  } else {
    ro.out16 = R.act;
  }
  if (R.row_group >= 4 && beam_steal_on()) ro.beam_ctr = beam_ctr.p;
  RET_IF(pa_decode_internal(&view, R.q, hid, R.o, R.beam_rows, R.ctx, R.n, H, D, cfg.max_seq_len,
                            cfg.attn_scale, pps, R.attn_ws, R.attn_ws_bytes, st, &ro,
                            R.row_group, plan));
  if (R.wgm_quant && !plan)  // the packed int8 o_proj input + row scales
    LLM_HIP_RET(launch_quantize_rows(R.o, R.n, hid, static_cast<int8_t*>(R.act), R.sa, st, 1));
  return LLM_OK;
}

int llm_decoder::layer_post(int l, hipStream_t st, const Rows& R) {
  const size_t lh = (size_t)l * hid;
  const bool i8 = wdtype == LLM_I8;
  WeightGemm g;
  g.dtype = wdtype;
  g.a_packed = 1;
  g.w_keep = w_keep;
  g.A = R.act;
  g.M = R.n;
  // o_proj: input produced (packed) by the attention merge, or quantised from
  // the attention's fp32 rows by the GEMM's own prologue
  g.W_packed = wo.p + sz_o * l; g.N = hid; g.K = hid; g.C = R.x;
  if (i8) { g.sa = R.sa; g.sw = sw_o.p + lh; }
  const bool qpro = quant_prologue(R);
  if (qpro) {
    g.ln_x = R.o;
    g.ln_quant_only = 1;
    if (tap_q) { g.act_out = R.act; g.sa_out = R.sa; }  // the taps read A and the scales back
  }
  if (!R.oacc) RET_IF(weight_gemm(g, st));  // (fused: the attention wrote x)
  g.ln_x = nullptr; g.ln_quant_only = 0; g.act_out = nullptr; g.sa_out = nullptr;
  RET_IF(tap(l, 1, R, hid, st));
  // LN2 -> mlp_fc1 (+b1, ReLU)
  const bool split_fc2 = fc2_split(R);
  RET_IF(layer_norm_into(g, R, ln2_g.p + lh, ln2_b.p + lh, st, split_fc2 ? R.x : nullptr));
  g.W_packed = w1.p + sz_1 * l; g.N = inter; g.K = hid;
  g.bias = b1.p + (size_t)l * inter; g.act = LLM_ACT_RELU;
  if (i8) {
    g.C = R.h1;
    g.sw = sw1.p + (size_t)l * inter;
  } else {
    // fp16 decoder: the fc1 epilogue writes fc2's packed fp16 input directly
    // (no per-row scale to wait for, so no conversion launch)
    g.C = nullptr;
    g.C16 = R.act2;
  }
  RET_IF(weight_gemm(g, st));
  RET_IF(tap(l, 2, R, hid, st));
  g.ln_x = nullptr; g.ln_emb = nullptr; g.act_out = nullptr; g.sa_out = nullptr;
  g.C16 = nullptr;
  if (!i8) g.A = R.act2;
  // quantise h1 -> mlp_fc2 (+b2)
  if (i8)
    LLM_HIP_RET(launch_quantize_rows(R.h1, R.n, inter, static_cast<int8_t*>(R.act), R.sa, st, 1));
  RET_IF(tap(l, 3, R, inter, st));
  g.W_packed = w2.p + sz_2 * l; g.N = hid; g.K = inter; g.C = R.x;
  g.bias = b2.p + lh; g.act = LLM_ACT_NONE;
  if (i8) g.sw = sw2.p + lh;
  g.ksplit2 = split_fc2 ? 1 : 0;  // (x was zeroed by the LN2 launch)
  return weight_gemm(g, st);
}

// Rows r0 .. r0 + n - 1 of the decode-step buffers.
Rows llm_decoder::step_rows(int r0, int n, uint8_t* ws) {
  Rows R;
  R.n = n;
  R.x = x.p + (size_t)r0 * hid;
  R.q = qkv.p + (size_t)r0 * hid;
  R.o = o.p + (size_t)r0 * hid;
  R.h1 = h1.p + (size_t)r0 * inter;
  R.act = wdtype == LLM_I8 ? (void*)(qa.p + (size_t)r0 * qa_ld) : (void*)(a16.p + (size_t)r0 * qa_ld);
  if (wdtype == LLM_F16) R.act2 = a16.p + (b16 + (size_t)r0) * qa_ld;
  R.sa = sa.p + r0;
  R.pos = pos.p + r0;
  R.ctx = ctx.p + r0;
  R.table_row0 = r0;
  R.row_group = r0 % row_group == 0 ? row_group : 1;
  R.attn_ws = ws;
  R.attn_ws_bytes = attn_ws_bytes;
  return R;
}

// Tap stage `stage` of layer l (0: LN1 out, 1: attention out, 2: LN2 out,
// 3: fc1 out): the rows' packed int8 activations (K per row) and row scales.
// Decode rows only (prefill chunks are not tapped); captured into the graph.
// FP16 decoders: the four packed fp16 GEMM inputs (2 bytes per element, no
// scales); stage 3 (fc2's input) is act2, written by the fc1 epilogue.
int llm_decoder::tap(int l, int stage, const Rows& R, int K, hipStream_t st) {
  if (!tap_q || R.prefill_row >= 0 || R.beam_rows) return LLM_OK;
  const bool f16 = wdtype == LLM_F16;
  const size_t es = f16 ? 2 : 1;
  const size_t slot = (size_t)l * 4 + stage;
  const size_t n16 = ((size_t)R.n + 15) / 16 * 16;
  const size_t r0 = (size_t)R.table_row0;  // rows r0.. of the step (16-row aligned)
  const void* src = f16 && stage == 3 ? R.act2 : R.act;
  LLM_HIP_RET(hipMemcpyAsync(tap_q + (slot * b16 * qa_ld + r0 * K) * es, src, n16 * K * es,
                             hipMemcpyDeviceToDevice, st));
  if (!f16)
    LLM_HIP_RET(hipMemcpyAsync(tap_s + slot * maxB + r0, R.sa, sizeof(float) * R.n,
                               hipMemcpyDeviceToDevice, st));
  return LLM_OK;
}

// LM head + token choice for rows r0.. (x rows given): logits into the step's
// logits buffer; greedy ids from the LM head's fused argmax partials, or a
// device draw (sample_rows) with the rows' positions as draw counters.
// adv_pos / adv_ctx (optional): advance the rows' positions afterwards (fused
// into the argmax launch; a launch of its own after a draw, which reads them).
int llm_decoder::next_tokens(const float* xr, int n, int r0, const int32_t* ctr, hipStream_t st,
                             int32_t* adv_pos, int32_t* adv_ctx) {
  float* lg = logits.p + (size_t)r0 * V;
  const bool sample = temperature > 0.f && top_k != 1;
  float* pv = lm_pv.p + (size_t)r0 * lm_nwg;
  int32_t* pi = lm_pi.p + (size_t)r0 * lm_nwg;
  LLM_HIP_RET(launch_lm_head(xr, emb_packed.p, lg, n, V, hid, sample ? nullptr : pv, pi, st));
  if (sample) {
    LLM_HIP_RET(launch_sample(lg, n, r0, V, temperature, top_k, top_p, sample_seed, ctr,
                              tokens.p + r0, st));
    if (adv_pos) LLM_HIP_RET(launch_advance(adv_pos, adv_ctx, n, st));
  } else {
    LLM_HIP_RET(launch_argmax_partials(pv, pi, n, lm_nwg, tokens.p + r0, st, adv_pos, adv_ctx));
  }
  return LLM_OK;
}

// The step's embedding: no launch of its own; layer 0's first LayerNorm
// (launch or GEMM prologue) reads E[token] rows directly (embed_src).
int llm_decoder::step_head(hipStream_t st, int r0, int n) {
  (void)st;
  embed_src = LnSource{};
  embed_src.emb = reinterpret_cast<const _Float16*>(emb.p);
  embed_src.tok = tokens.p + r0;
  embed_src.V = V;
  (void)n;
  return LLM_OK;
}

int llm_decoder::step_tail(hipStream_t st, int r0, int n) {
  return next_tokens(x.p + (size_t)r0 * hid, n, r0, pos.p + r0, st, pos.p + r0, ctx.p + r0);
}

// One decode step of all active rows (captured into the step graph).
int llm_decoder::enqueue_step(hipStream_t st) {
  Rows R = step_rows(0, batch, attn_ws.p);
  if (oproj_fusable(R)) R.oacc = oacc.p, R.oproj_out = R.x, R.oflag = oflag.p;
  R.wgm_quant = wgm_quant_ok(R);
  RET_IF(step_head(st, 0, batch));
  for (int l = 0; l < L; ++l) {
    RET_IF(layer_pre(l, st, R));
    RET_IF(layer_attn(l, st, R));
    RET_IF(layer_post(l, st, R));
  }
  return step_tail(st, 0, batch);
}

int llm_decoder::run_step(const int32_t* tokens_host, float* logits_dev, int32_t* next_host,
                          hipStream_t st) {
  LLM_REQUIRE(weights_ready, "decoder: weights not loaded");
  LLM_REQUIRE(batch > 0, "decoder: no active rows (call generate / begin first)");
  KvCache* k = kv_impl(kv);
  {
    std::lock_guard<std::mutex> g(k->mu);
    for (int b = 0; b < batch; ++b) {
      LLM_REQUIRE(h_pos[b] < cfg.max_seq_len, "decoder: row reached max_seq_len");
      RET_IF(k->prepare_append(b, h_pos[b]));
    }
    RET_IF(k->sync(st));
  }
  if (tokens_host) {
    for (int b = 0; b < batch; ++b)
      LLM_REQUIRE(tokens_host[b] >= 0 && tokens_host[b] < V, "decoder: token id out of range");
    LLM_HIP_RET(hipMemcpyAsync(tokens.p, tokens_host, sizeof(int32_t) * batch,
                               hipMemcpyHostToDevice, st));
  }
  if (!use_graph) {
    RET_IF(enqueue_step(st));
  } else {
    if (graph_batch != batch) {
      if (graph) { (void)hipGraphExecDestroy(graph); graph = nullptr; }
      hipGraph_t g;
      LLM_HIP_RET(hipStreamSynchronize(st));
      LLM_HIP_RET(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
      int rc = enqueue_step(stream);
      hipError_t e = hipStreamEndCapture(stream, &g);
      if (rc) return rc;
      if (e != hipSuccess)
        return fail(LLM_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
      e = hipGraphInstantiate(&graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (e != hipSuccess)
        return fail(LLM_ERR_HIP, std::string("graph instantiate: ") + hipGetErrorString(e));
      graph_batch = batch;
    }
    LLM_HIP_RET(hipGraphLaunch(graph, st));
  }
  for (int b = 0; b < batch; ++b) h_pos[b] += 1;
  if (logits_dev)
    LLM_HIP_RET(hipMemcpyAsync(logits_dev, logits.p, sizeof(float) * batch * V,
                               hipMemcpyDeviceToDevice, st));
  if (next_host) {
    LLM_HIP_RET(hipMemcpyAsync(next_host, tokens.p, sizeof(int32_t) * batch,
                               hipMemcpyDeviceToHost, st));
    if (oflag.p) {
      hipLaunchKernelGGL(take_flag_kernel, dim3(1), dim3(1), 0, st, oflag.p);
      LLM_HIP_RET(hipGetLastError());
      LLM_HIP_RET(hipMemcpyAsync(h_oflag, oflag.p + 1, sizeof(int), hipMemcpyDeviceToHost, st));
    }
    LLM_HIP_RET(hipStreamSynchronize(st));
    if (oflag.p) return report_range(*h_oflag);
  }
  return LLM_OK;
}

// The fused o_proj's range guard (common.hpp oacc_term), reported ONCE: the
// flag is read and cleared in one device atomic (take_flag_kernel), so a
// clamp by a step still running on another stream is never lost between the
// read and the clear; a taken flag returns LLM_ERR_RANGE, and the steps after
// it (and the next llm_decoder_sync) succeed unless they clamp again.
// range_clamped keeps the fact for llm_decoder_oproj_status until the next
// begin / generate.  Caller holds mu; `flag` is take_flag_kernel's result.
int llm_decoder::report_range(int flag) {
  if (!flag) return LLM_OK;
  range_clamped = 1;
  return fail(LLM_ERR_RANGE,
              "decoder: a head product of the fused o_proj left its fixed-point range "
              "(|v| > (2^23 - 1) / num_heads, or not finite) and was clamped; the affected "
              "hidden values of that step are wrong");
}

int llm_decoder::oproj_range_status() {
  if (!oflag.p) return LLM_OK;
  int f = 0;
  hipLaunchKernelGGL(take_flag_kernel, dim3(1), dim3(1), 0, stream, oflag.p);
  LLM_HIP_RET(hipGetLastError());
  LLM_HIP_RET(hipMemcpyAsync(&f, oflag.p + 1, sizeof(int), hipMemcpyDeviceToHost, stream));
  LLM_HIP_RET(hipStreamSynchronize(stream));
  return report_range(f);
}

// Chunked prefill of `n` prompt tokens of active row `row` (the reference's
// is_prefill pass, attention/attention_cuda.hpp:21): the chunk's tokens are
// the rows of one layer pass — M = chunk-size weight GEMMs, the K/V of every
// token appended to the row's pages by the qkv epilogue, and causal attention
// through the same paged decode kernel (token i of the chunk attends to the
// row's positions < p0 + i + 1 via beam_ids = row, context_lens = p0 + i + 1).
// The last token's logits pick the row's next token (argmax / sampling), so
// decode steps continue from the prompt.
int llm_decoder::prefill(int row, const int32_t* toks, int n, hipStream_t st) {
  LLM_REQUIRE(weights_ready, "prefill: weights not loaded");
  LLM_REQUIRE(row >= 0 && row < batch, "prefill: row is not active");
  LLM_REQUIRE(n >= 1 && toks, "prefill: need >= 1 token");
  LLM_REQUIRE(h_pos[row] + n < cfg.max_seq_len, "prefill: prompt exceeds max_seq_len");
  for (int i = 0; i < n; ++i) LLM_REQUIRE(toks[i] >= 0 && toks[i] < V, "prefill: token id out of range");
  const int C = std::min(n, kPrefillChunk);
  if (C > pf_cap) {
    const size_t C16 = ((size_t)C + 15) / 16 * 16;
    RET_IF(px.alloc((size_t)C * hid));
    RET_IF(pq.alloc((size_t)C * hid));
    RET_IF(po.alloc((size_t)C * hid));
    RET_IF(ph1.alloc((size_t)C * inter));
    RET_IF(psa.alloc((size_t)C));
    RET_IF(pact.alloc(C16 * std::max(hid, inter) * (wdtype == LLM_I8 ? 1 : 4)));  // F16: act, act2
    RET_IF(pmeta.alloc((size_t)4 * C));
    pws_bytes = 16;
    for (int b = 1; b <= C; ++b)
      pws_bytes = std::max(pws_bytes, pa_decode_workspace_bytes(b, H, D, max_tiles, 0));
    {  // the MFMA prefill's split partials (its split count is bounded at any p0)
      pa_kv_view v0;
      RET_IF(kv_cache_view(kv, 0, &v0));
      for (int b = 1; b <= C; ++b)
        pws_bytes = std::max(pws_bytes, pa_prefill_ws_bytes(&v0, cfg.max_seq_len - b, b));
    }
    RET_IF(pws.alloc(pws_bytes));
    pf_cap = C;
  }
  KvCache* k = kv_impl(kv);
  std::vector<int32_t> meta((size_t)4 * C), pc(2);
  for (int c0 = 0; c0 < n; c0 += C) {
    const int m = std::min(C, n - c0);
    const int p0 = h_pos[row];
    {
      std::lock_guard<std::mutex> gk(k->mu);
      for (int t = p0; t < p0 + m; t = (t / TS + 1) * TS) RET_IF(k->prepare_append(row, t));
      RET_IF(k->sync(st));
    }
    for (int i = 0; i < m; ++i) {
      meta[i] = p0 + i;
      meta[C + i] = p0 + i + 1;
      meta[2 * C + i] = row;
      meta[3 * C + i] = toks[c0 + i];
    }
    LLM_HIP_RET(hipMemcpyAsync(pmeta.p, meta.data(), meta.size() * sizeof(int32_t),
                               hipMemcpyHostToDevice, st));
    Rows R;
    R.n = m;
    R.x = px.p; R.q = pq.p; R.o = po.p; R.h1 = ph1.p; R.act = pact.p; R.sa = psa.p;
    if (wdtype == LLM_F16)
      R.act2 = pact.p + (((size_t)C + 15) / 16 * 16) * std::max(hid, inter) * 2;
    R.pos = pmeta.p; R.ctx = pmeta.p + C; R.beam_rows = pmeta.p + 2 * C;
    R.prefill_row = row;
    R.prefill_p0 = p0;
    R.attn_ws = pws.p; R.attn_ws_bytes = pws_bytes;
    LLM_HIP_RET(launch_embed(emb.p, pmeta.p + 3 * C, m, hid, V, px.p, st));
    embed_src = LnSource{};  // (a failed step enqueue could have left it set)
    for (int l = 0; l < L; ++l) {
      RET_IF(layer_pre(l, st, R));
      RET_IF(layer_attn(l, st, R));
      RET_IF(layer_post(l, st, R));
    }
    h_pos[row] = p0 + m;
    if (c0 + m == n) {  // last token: logits -> the row's next token, decode state
      RET_IF(next_tokens(px.p + (size_t)(m - 1) * hid, 1, row, pmeta.p + (m - 1), st));
      pc[0] = p0 + m;
      pc[1] = p0 + m + 1;
      LLM_HIP_RET(hipMemcpyAsync(pos.p + row, &pc[0], sizeof(int32_t), hipMemcpyHostToDevice, st));
      LLM_HIP_RET(hipMemcpyAsync(ctx.p + row, &pc[1], sizeof(int32_t), hipMemcpyHostToDevice, st));
    }
    LLM_HIP_RET(hipStreamSynchronize(st));  // meta / pc staging reused next chunk
  }
  return LLM_OK;
}

static int reset_rows(llm_decoder* d, int batch, int start_pos) {
  LLM_REQUIRE(batch > 0 && batch <= d->maxB, "decoder: batch must be in [1, max_batch]");
  RET_IF(kv_cache_clear(d->kv));
  d->batch = batch;
  if (d->row_group != 1) d->graph_batch = -1;  // the captured attention launch used the beam group
  d->row_group = 1;
  d->h_pos.assign(d->maxB, 0);
  for (int b = 0; b < batch; ++b) d->h_pos[b] = start_pos;
  if (d->oacc.p) LLM_HIP_RET(hipMemset(d->oacc.p, 0, sizeof(long long) * d->oacc.n));
  if (d->oflag.p) LLM_HIP_RET(hipMemset(d->oflag.p, 0, sizeof(int)));
  d->range_clamped = 0;
  std::vector<int32_t> pos(batch, start_pos), ctx(batch, start_pos + 1), tok(batch, 0);
  LLM_HIP_RET(hipMemcpy(d->pos.p, pos.data(), sizeof(int32_t) * batch, hipMemcpyHostToDevice));
  LLM_HIP_RET(hipMemcpy(d->ctx.p, ctx.data(), sizeof(int32_t) * batch, hipMemcpyHostToDevice));
  LLM_HIP_RET(hipMemcpy(d->tokens.p, tok.data(), sizeof(int32_t) * batch, hipMemcpyHostToDevice));
  LLM_HIP_RET(hipDeviceSynchronize());
  return LLM_OK;
}

extern "C" int llm_decoder_begin_synthetic(llm_decoder* d, int batch, int context_len,
                                           uint64_t seed, int shuffle) {
  LLM_REQUIRE(d, "llm_decoder_begin_synthetic: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_REQUIRE(context_len >= 0 && context_len < d->cfg.max_seq_len,
              "llm_decoder_begin_synthetic: context_len must be in [0, max_seq_len)");
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  RET_IF(reset_rows(d, batch, context_len));
  KvCache* k = kv_impl(d->kv);
  {
    std::lock_guard<std::mutex> gk(k->mu);
    if (shuffle) {  // non-contiguous page gather (shuffled page pool, seed 7)
      std::mt19937_64 rng(seed ^ 7);
      for (auto& f : k->free_lists) std::shuffle(f.begin(), f.end(), rng);
    }
  }
  for (int b = 0; b < batch; ++b) RET_IF(kv_cache_reserve(d->kv, b, context_len));
  RET_IF(kv_cache_sync(d->kv, d->stream));
  // seeded random fp16 K/V over the whole pools (K scaled so q.k ~ O(1))
  const size_t np = (size_t)k->num_pages, pe = k->page_elems, ps = k->page_stride() / k->es;
  LLM_HIP_RET(launch_fill_random_f16(k->k_pool, np, pe, ps, seed * 2 + 1, 0.05f, d->stream));
  LLM_HIP_RET(launch_fill_random_f16(k->v_pool, np, pe, ps, seed * 2 + 2, 1.0f, d->stream));
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  return LLM_OK;
}

extern "C" int llm_decoder_begin_beams(llm_decoder* d, int num_seqs, int beam_width,
                                       int shared_len, int beam_len, uint64_t seed, int shuffle) {
  LLM_REQUIRE(d, "llm_decoder_begin_beams: NULL");
  LLM_REQUIRE(num_seqs > 0 && beam_width >= 1 && beam_width <= 4 && shared_len >= 0 &&
                  beam_len >= 0,
              "llm_decoder_begin_beams: bad arguments (beam_width in [1, 4])");
  std::lock_guard<std::mutex> g(d->mu);
  const int ctx_len = shared_len + beam_len;
  LLM_REQUIRE(ctx_len < d->cfg.max_seq_len,
              "llm_decoder_begin_beams: shared_len + beam_len must be < max_seq_len");
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  const int batch = num_seqs * beam_width;
  RET_IF(reset_rows(d, batch, ctx_len));
  KvCache* k = kv_impl(d->kv);
  if (shuffle) {
    std::lock_guard<std::mutex> gk(k->mu);
    std::mt19937_64 rng(seed ^ 7);
    for (auto& f : k->free_lists) std::shuffle(f.begin(), f.end(), rng);
  }
  // beam 0 of each sequence owns the shared prefix; the other beams fork its
  // page table (shared pages, refcounted) and then get private pages for their
  // own beam_len tokens.
  for (int sq = 0; sq < num_seqs; ++sq) {
    const int b0 = sq * beam_width;
    RET_IF(kv_cache_reserve(d->kv, b0, shared_len));
    for (int w = 1; w < beam_width; ++w) RET_IF(kv_cache_fork(d->kv, b0, b0 + w));
    for (int w = 0; w < beam_width; ++w) RET_IF(kv_cache_reserve(d->kv, b0 + w, ctx_len));
  }
  RET_IF(kv_cache_sync(d->kv, d->stream));
  const size_t np = (size_t)k->num_pages, pe = k->page_elems, ps = k->page_stride() / k->es;
  LLM_HIP_RET(launch_fill_random_f16(k->k_pool, np, pe, ps, seed * 2 + 1, 0.05f, d->stream));
  LLM_HIP_RET(launch_fill_random_f16(k->v_pool, np, pe, ps, seed * 2 + 2, 1.0f, d->stream));
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  d->row_group = beam_width;
  d->graph_batch = -1;  // re-capture: the attention launch depends on row_group
  return LLM_OK;
}

extern "C" int llm_decoder_prefill(llm_decoder* d, int row, const int32_t* tokens, int n) {
  LLM_REQUIRE(d, "llm_decoder_prefill: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  return d->prefill(row, tokens, n, d->stream);
}

extern "C" int llm_decoder_set_sampling(llm_decoder* d, float temperature, int top_k, float top_p,
                                        uint64_t seed) {
  LLM_REQUIRE(d, "llm_decoder_set_sampling: NULL");
  LLM_REQUIRE(top_k >= 0 && top_p > 0.f && top_p <= 1.f && d->V <= 65536,
              "llm_decoder_set_sampling: top_k >= 0, 0 < top_p <= 1, vocab <= 65536");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  d->temperature = temperature;
  d->top_k = top_k;
  d->top_p = top_p;
  d->sample_seed = seed;
  d->graph_batch = -1;  // the step graph changes
  return LLM_OK;
}

extern "C" int llm_decoder_set_taps(llm_decoder* d, int8_t* q_dev, float* s_dev) {
  LLM_REQUIRE(d, "llm_decoder_set_taps: NULL");
  LLM_REQUIRE((q_dev == nullptr) == (s_dev == nullptr),
              "llm_decoder_set_taps: give both tap buffers or neither");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  d->tap_q = q_dev;
  d->tap_s = s_dev;
  d->graph_batch = -1;  // the step graph gains / loses the tap copies
  return LLM_OK;
}

extern "C" int llm_decoder_attention_plan(llm_decoder* d, int* nsplit, int* form) {
  LLM_REQUIRE(d && nsplit && form, "llm_decoder_attention_plan: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_REQUIRE(d->batch > 0, "llm_decoder_attention_plan: no active rows");
  Rows R = d->step_rows(0, d->batch, d->attn_ws.p);
  if (d->oproj_fusable(R)) R.oacc = d->oacc.p, R.oproj_out = R.x, R.oflag = d->oflag.p;
  R.wgm_quant = d->wgm_quant_ok(R);
  PaPlan p;
  RET_IF(d->layer_attn(0, d->stream, R, &p));
  *nsplit = p.nsplit;
  *form = p.form;
  return LLM_OK;
}

extern "C" int llm_decoder_run_attention(llm_decoder* d, int layer, void* stream) {
  LLM_REQUIRE(d, "llm_decoder_run_attention: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_REQUIRE(d->batch > 0, "llm_decoder_run_attention: no active rows");
  LLM_REQUIRE(layer >= 0 && layer < d->L, "llm_decoder_run_attention: layer out of range");
  hipStream_t st = stream ? as_stream(stream) : d->stream;
  Rows R = d->step_rows(0, d->batch, d->attn_ws.p);
  // the step's fused o_proj writes the attention rows' fp32 buffer here, not
  // x, and accumulates into columns of its own (oacc_run: zero at allocation,
  // and every completed column clears itself, as the step's do) with a range
  // flag of its own (oflag_run: a clamp here never fails a step or a sync)
  if (d->oproj_fusable(R)) {
    if (!d->oacc_run.p) {
      RET_IF(d->oacc_run.alloc(d->oacc.n));
      LLM_HIP_RET(hipMemset(d->oacc_run.p, 0, sizeof(long long) * d->oacc_run.n));
      RET_IF(d->oflag_run.alloc(1));
      LLM_HIP_RET(hipMemset(d->oflag_run.p, 0, sizeof(int)));
    }
    R.oacc = d->oacc_run.p, R.oproj_out = R.o, R.oflag = d->oflag_run.p;
  }
  R.wgm_quant = d->wgm_quant_ok(R);
  return d->layer_attn(layer, st, R);
}

extern "C" int llm_decoder_oproj_status(llm_decoder* d, int* clamped, long long* nonzero_columns) {
  LLM_REQUIRE(d, "llm_decoder_oproj_status: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_HIP_RET(hipDeviceSynchronize());
  int f = 0;
  long long nz = 0;
  if (d->oflag.p) LLM_HIP_RET(hipMemcpy(&f, d->oflag.p, sizeof(int), hipMemcpyDeviceToHost));
  f = f || d->range_clamped;
  for (const DevBuf<long long>* b : {&d->oacc, &d->oacc_run}) {
    if (!b->p) continue;
    std::vector<long long> h(b->n);
    LLM_HIP_RET(hipMemcpy(h.data(), b->p, sizeof(long long) * b->n, hipMemcpyDeviceToHost));
    for (long long v : h) nz += v != 0;
  }
  if (clamped) *clamped = f;
  if (nonzero_columns) *nonzero_columns = nz;
  return LLM_OK;
}

extern "C" int llm_decoder_step(llm_decoder* d, const int32_t* tokens, float* logits_dev,
                                int32_t* next_host, void* stream) {
  LLM_REQUIRE(d, "llm_decoder_step: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  hipStream_t st = stream ? as_stream(stream) : d->stream;
  return d->run_step(tokens, logits_dev, next_host, st);
}

extern "C" int llm_decoder_copy_next(llm_decoder* d, int32_t* dst_dev, void* stream) {
  LLM_REQUIRE(d && dst_dev, "llm_decoder_copy_next: NULL");
  std::lock_guard<std::mutex> g(d->mu);
  LLM_REQUIRE(d->batch > 0, "llm_decoder_copy_next: no active rows");
  hipStream_t st = stream ? as_stream(stream) : d->stream;
  LLM_HIP_RET(hipMemcpyAsync(dst_dev, d->tokens.p, sizeof(int32_t) * d->batch,
                             hipMemcpyDeviceToDevice, st));
  return LLM_OK;
}

extern "C" int llm_decoder_sync(llm_decoder* d) {
  LLM_REQUIRE(d, "llm_decoder_sync: NULL");
  LLM_HIP_RET(hipDeviceSynchronize());
  std::lock_guard<std::mutex> g(d->mu);
  return d->oproj_range_status();
}

extern "C" int llm_decoder_context_len(const llm_decoder* d, int row) {
  if (!d || row < 0 || row >= d->batch) return -1;
  return d->h_pos[row];
}

extern "C" int llm_decoder_generate(llm_decoder* d, const int32_t* prompts,
                                    const int32_t* prompt_lens, int prompt_stride, int batch,
                                    int max_gen_len, float temperature, int32_t* out) {
  LLM_REQUIRE(d && prompts && prompt_lens && out, "llm_decoder_generate: NULL");
  LLM_REQUIRE(max_gen_len >= 0, "llm_decoder_generate: max_gen_len < 0");
  // generate is greedy argmax whatever the temperature, as the reference's
  // sample_from_logits (decoder/cuda_decoder.cu:7-14): argmax is invariant to
  // temperature > 0.  A device-sampling mode set by llm_decoder_set_sampling
  // applies to llm_decoder_step only; it is suspended here and restored after.
  (void)temperature;
  std::lock_guard<std::mutex> g(d->mu);
  struct SamplingGuard {
    llm_decoder* d;
    float t;
    bool active;
    explicit SamplingGuard(llm_decoder* dd)
        : d(dd), t(dd->temperature), active(dd->temperature > 0.f && dd->top_k != 1) {
      if (active) { d->temperature = 0.f; d->graph_batch = -1; }
    }
    ~SamplingGuard() {
      if (active) { d->temperature = t; d->graph_batch = -1; }
    }
  } sampling_guard(d);
  LLM_REQUIRE(batch >= 1 && batch <= d->maxB, "llm_decoder_generate: batch out of range");
  int max_len = 0;
  for (int b = 0; b < batch; ++b) {
    LLM_REQUIRE(prompt_lens[b] >= 1 && prompt_lens[b] <= prompt_stride,
                "llm_decoder_generate: every prompt needs >= 1 token");
    for (int i = 0; i < prompt_lens[b]; ++i) {
      const int t = prompts[(size_t)b * prompt_stride + i];
      LLM_REQUIRE(t >= 0 && t < d->V, "llm_decoder_generate: token id out of range");
    }
    max_len = std::max(max_len, prompt_lens[b]);
  }
  if (max_gen_len == 0) return LLM_OK;
  LLM_REQUIRE(max_len + max_gen_len - 1 <= d->cfg.max_seq_len,
              "llm_decoder_generate: prompt + max_gen_len exceeds max_seq_len");
  LLM_HIP_RET(hipStreamSynchronize(d->stream));
  RET_IF(reset_rows(d, batch, 0));
  // every prompt but its last token goes through chunked prefill; decode steps
  // then run all rows in lockstep, each at its own position
  for (int b = 0; b < batch; ++b)
    if (prompt_lens[b] > 1)
      RET_IF(d->prefill(b, prompts + (size_t)b * prompt_stride, prompt_lens[b] - 1, d->stream));
  // a step whose fused o_proj clamped (LLM_ERR_RANGE) still produced its ids:
  // generation runs to the end, fills `out`, and then returns the status
  std::vector<int32_t> tok(batch), next(batch);
  int range_rc = LLM_OK;
  for (int s = 0; s < max_gen_len; ++s) {
    for (int b = 0; b < batch; ++b)
      tok[b] = s == 0 ? prompts[(size_t)b * prompt_stride + prompt_lens[b] - 1] : next[b];
    const int rc = d->run_step(tok.data(), nullptr, next.data(), d->stream);
    if (rc == LLM_ERR_RANGE) range_rc = rc;
    else RET_IF(rc);
    for (int b = 0; b < batch; ++b) out[(size_t)b * max_gen_len + s] = next[b];
  }
  if (range_rc) return fail(LLM_ERR_RANGE, "llm_decoder_generate: the fused o_proj clamped a head "
                                           "product in at least one step; `out` is complete, the "
                                           "ids after that step may differ");
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// weight files (weights/README.md:26-38; raw little-endian .bin)
// ---------------------------------------------------------------------------
static int read_file(const std::string& path, std::vector<char>& buf, size_t expect) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) return fail(LLM_ERR_IO, "cannot open weight file: " + path);  // decoder_block.hpp:13-15
  const size_t size = (size_t)f.tellg();
  if (expect && size != expect)
    return fail(LLM_ERR_IO, path + ": expected " + std::to_string(expect) + " bytes, found " +
                                std::to_string(size));
  buf.resize(size);
  f.seekg(0);
  f.read(buf.data(), size);
  if (!f) return fail(LLM_ERR_IO, "failed to read from file: " + path);
  return LLM_OK;
}

static int write_file(const std::string& path, const void* p, size_t n) {
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, "cannot create " + path);
  f.write(static_cast<const char*>(p), n);
  if (!f) return fail(LLM_ERR_IO, "write failed: " + path);
  return LLM_OK;
}

static uint16_t f32_to_f16_bits(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

// fp32 directory (CUDADecoder::load_weights): embedding.bin [V][hid];
// layer_i/{ln1.bin, ln2.bin} gamma+beta; attn_wq/wk/wv/wo.bin [hid][hid];
// mlp_fc1.bin [hid][inter]; mlp_fc2.bin [inter][hid]; mlp_biases.bin [inter+hid].
struct Fp32Model {
  std::vector<float> emb, ln1, ln2, wqkv, wo, w1, w2, b1, b2;  // ln: [L][2][hid]
};

static int load_fp32_dir(const std::string& dir, int L, int hid, int inter, int V, Fp32Model& m) {
  std::vector<char> buf;
  auto rd = [&](const std::string& p, size_t n, float* dst) -> int {
    RET_IF(read_file(p, buf, n * 4));
    std::memcpy(dst, buf.data(), n * 4);
    return LLM_OK;
  };
  m.emb.resize((size_t)V * hid);
  RET_IF(rd(dir + "/embedding.bin", m.emb.size(), m.emb.data()));
  m.ln1.resize((size_t)L * 2 * hid); m.ln2.resize((size_t)L * 2 * hid);
  m.wqkv.resize((size_t)L * hid * 3 * hid); m.wo.resize((size_t)L * hid * hid);
  m.w1.resize((size_t)L * hid * inter); m.w2.resize((size_t)L * inter * hid);
  m.b1.resize((size_t)L * inter); m.b2.resize((size_t)L * hid);
  std::vector<float> tmp((size_t)hid * hid), bias(inter + hid);
  for (int l = 0; l < L; ++l) {
    const std::string p = dir + "/layer_" + std::to_string(l);
    RET_IF(rd(p + "/ln1.bin", 2 * hid, m.ln1.data() + (size_t)l * 2 * hid));
    RET_IF(rd(p + "/ln2.bin", 2 * hid, m.ln2.data() + (size_t)l * 2 * hid));
    const char* names[3] = {"/attn_wq.bin", "/attn_wk.bin", "/attn_wv.bin"};
    for (int j = 0; j < 3; ++j) {  // fuse q|k|v column blocks: Wqkv[k][j*hid + n]
      RET_IF(rd(p + names[j], (size_t)hid * hid, tmp.data()));
      float* dst = m.wqkv.data() + (size_t)l * hid * 3 * hid;
      for (int k = 0; k < hid; ++k)
        std::memcpy(dst + (size_t)k * 3 * hid + (size_t)j * hid, tmp.data() + (size_t)k * hid,
                    hid * 4);
    }
    RET_IF(rd(p + "/attn_wo.bin", (size_t)hid * hid, m.wo.data() + (size_t)l * hid * hid));
    RET_IF(rd(p + "/mlp_fc1.bin", (size_t)hid * inter, m.w1.data() + (size_t)l * hid * inter));
    RET_IF(rd(p + "/mlp_fc2.bin", (size_t)inter * hid, m.w2.data() + (size_t)l * inter * hid));
    RET_IF(rd(p + "/mlp_biases.bin", (size_t)inter + hid, bias.data()));
    std::memcpy(m.b1.data() + (size_t)l * inter, bias.data(), (size_t)inter * 4);
    std::memcpy(m.b2.data() + (size_t)l * hid, bias.data() + inter, (size_t)hid * 4);
  }
  return LLM_OK;
}

static void split_ln(const std::vector<float>& ln, int L, int hid, std::vector<float>& g,
                     std::vector<float>& b) {
  g.resize((size_t)L * hid);
  b.resize((size_t)L * hid);
  for (int l = 0; l < L; ++l) {
    std::memcpy(g.data() + (size_t)l * hid, ln.data() + (size_t)l * 2 * hid, hid * 4);
    std::memcpy(b.data() + (size_t)l * hid, ln.data() + (size_t)l * 2 * hid + hid, hid * 4);
  }
}

// Per-output-column int8 quantisation (int8_quant.cpp semantics, one scale per column).
static void quantize_cols(const float* w, int K, int N, int8_t* q, float* inv) {
  for (int n = 0; n < N; ++n) {
    float mn = w[n], mx = w[n];
    for (int k = 1; k < K; ++k) {
      mn = std::min(mn, w[(size_t)k * N + n]);
      mx = std::max(mx, w[(size_t)k * N + n]);
    }
    const float absmax = std::max(std::fabs(mn), std::fabs(mx));
    const float scale = 127.f / (absmax + 1e-6f);
    for (int k = 0; k < K; ++k) {
      int v = (int)std::round(w[(size_t)k * N + n] * scale);
      v = std::max(-128, std::min(127, v));
      q[(size_t)k * N + n] = (int8_t)v;
    }
    inv[n] = 1.0f / scale;
  }
}

extern "C" int llm_decoder_load_weights(llm_decoder* d, const char* dir) {
  LLM_REQUIRE(d && dir, "llm_decoder_load_weights: NULL");
  const int L = d->L, hid = d->hid, inter = d->inter, V = d->V;
  Fp32Model m;
  RET_IF(load_fp32_dir(dir, L, hid, inter, V, m));
  std::vector<float> g1, be1, g2, be2;
  split_ln(m.ln1, L, hid, g1, be1);
  split_ln(m.ln2, L, hid, g2, be2);
  std::vector<uint16_t> emb(m.emb.size());
  for (size_t i = 0; i < emb.size(); ++i) emb[i] = f32_to_f16_bits(m.emb[i]);
  if (d->wdtype == LLM_F16) {
    auto cvt = [](const std::vector<float>& s) {
      std::vector<uint16_t> o(s.size());
      for (size_t i = 0; i < s.size(); ++i) o[i] = f32_to_f16_bits(s[i]);
      return o;
    };
    auto qkv = cvt(m.wqkv), wo = cvt(m.wo), w1 = cvt(m.w1), w2 = cvt(m.w2);
    llm_f16_weights w{emb.data(), g1.data(), be1.data(), g2.data(), be2.data(), qkv.data(),
                      wo.data(), w1.data(), w2.data(), m.b1.data(), m.b2.data()};
    return llm_decoder_set_f16_weights(d, &w);
  }
  // INT8 decoder given fp32 weights: quantise on load
  std::vector<int8_t> qqkv(m.wqkv.size()), qo(m.wo.size()), q1(m.w1.size()), q2(m.w2.size());
  std::vector<float> sqkv((size_t)L * 3 * hid), so((size_t)L * hid), s1((size_t)L * inter),
      s2((size_t)L * hid);
  for (int l = 0; l < L; ++l) {
    quantize_cols(m.wqkv.data() + (size_t)l * hid * 3 * hid, hid, 3 * hid,
                  qqkv.data() + (size_t)l * hid * 3 * hid, sqkv.data() + (size_t)l * 3 * hid);
    quantize_cols(m.wo.data() + (size_t)l * hid * hid, hid, hid, qo.data() + (size_t)l * hid * hid,
                  so.data() + (size_t)l * hid);
    quantize_cols(m.w1.data() + (size_t)l * hid * inter, hid, inter,
                  q1.data() + (size_t)l * hid * inter, s1.data() + (size_t)l * inter);
    quantize_cols(m.w2.data() + (size_t)l * inter * hid, inter, hid,
                  q2.data() + (size_t)l * inter * hid, s2.data() + (size_t)l * hid);
  }
  llm_int8_weights w{emb.data(), g1.data(), be1.data(), g2.data(), be2.data(), qqkv.data(),
                     sqkv.data(), qo.data(), so.data(), q1.data(), s1.data(), m.b1.data(),
                     q2.data(), s2.data(), m.b2.data()};
  return llm_decoder_set_int8_weights(d, &w);
}

// INT8 directory written by llm_quantize_weights: embedding.f16 [V][hid] fp16;
// layer_i/{ln1.bin, ln2.bin (fp32 gamma+beta), attn_wqkv.i8 [hid][3hid],
// attn_wqkv.scale [3hid], attn_wo.i8/.scale, mlp_fc1.i8/.scale, mlp_fc2.i8/.scale,
// mlp_biases.bin [inter+hid] fp32}.
extern "C" int llm_quantize_weights(const char* fp32_dir, const char* int8_dir, int num_layers,
                                    int hidden_dim, int inter_dim, int vocab_size) {
  LLM_REQUIRE(fp32_dir && int8_dir && num_layers > 0 && hidden_dim > 0 && vocab_size > 0,
              "llm_quantize_weights: bad arguments");
  const int L = num_layers, hid = hidden_dim, inter = inter_dim > 0 ? inter_dim : 4 * hidden_dim;
  Fp32Model m;
  RET_IF(load_fp32_dir(fp32_dir, L, hid, inter, vocab_size, m));
  const std::string out = int8_dir;
  std::vector<uint16_t> emb(m.emb.size());
  for (size_t i = 0; i < emb.size(); ++i) emb[i] = f32_to_f16_bits(m.emb[i]);
  if (std::system(("mkdir -p '" + out + "'").c_str()) != 0)
    return fail(LLM_ERR_IO, "cannot create " + out);
  RET_IF(write_file(out + "/embedding.f16", emb.data(), emb.size() * 2));
  for (int l = 0; l < L; ++l) {
    const std::string p = out + "/layer_" + std::to_string(l);
    if (std::system(("mkdir -p '" + p + "'").c_str()) != 0)
      return fail(LLM_ERR_IO, "cannot create " + p);
    RET_IF(write_file(p + "/ln1.bin", m.ln1.data() + (size_t)l * 2 * hid, (size_t)2 * hid * 4));
    RET_IF(write_file(p + "/ln2.bin", m.ln2.data() + (size_t)l * 2 * hid, (size_t)2 * hid * 4));
    struct { const char* name; const float* w; int K, N; } mats[4] = {
        {"attn_wqkv", m.wqkv.data() + (size_t)l * hid * 3 * hid, hid, 3 * hid},
        {"attn_wo", m.wo.data() + (size_t)l * hid * hid, hid, hid},
        {"mlp_fc1", m.w1.data() + (size_t)l * hid * inter, hid, inter},
        {"mlp_fc2", m.w2.data() + (size_t)l * inter * hid, inter, hid}};
    for (auto& mt : mats) {
      std::vector<int8_t> q((size_t)mt.K * mt.N);
      std::vector<float> s(mt.N);
      quantize_cols(mt.w, mt.K, mt.N, q.data(), s.data());
      RET_IF(write_file(p + "/" + mt.name + ".i8", q.data(), q.size()));
      RET_IF(write_file(p + "/" + mt.name + ".scale", s.data(), s.size() * 4));
    }
    std::vector<float> bias(inter + hid);
    std::memcpy(bias.data(), m.b1.data() + (size_t)l * inter, (size_t)inter * 4);
    std::memcpy(bias.data() + inter, m.b2.data() + (size_t)l * hid, (size_t)hid * 4);
    RET_IF(write_file(p + "/mlp_biases.bin", bias.data(), bias.size() * 4));
  }
  return LLM_OK;
}

extern "C" int llm_decoder_load_quantized_weights(llm_decoder* d, const char* dir) {
  LLM_REQUIRE(d && dir, "llm_decoder_load_quantized_weights: NULL");
  LLM_REQUIRE(d->wdtype == LLM_I8, "llm_decoder_load_quantized_weights: decoder is not INT8");
  const int L = d->L, hid = d->hid, inter = d->inter, V = d->V;
  const std::string root = dir;
  std::vector<char> buf;
  std::vector<uint16_t> emb((size_t)V * hid);
  RET_IF(read_file(root + "/embedding.f16", buf, emb.size() * 2));
  std::memcpy(emb.data(), buf.data(), emb.size() * 2);
  std::vector<float> g1((size_t)L * hid), be1((size_t)L * hid), g2((size_t)L * hid), be2((size_t)L * hid);
  std::vector<int8_t> qqkv((size_t)L * hid * 3 * hid), qo((size_t)L * hid * hid),
      q1((size_t)L * hid * inter), q2((size_t)L * inter * hid);
  std::vector<float> sqkv((size_t)L * 3 * hid), so((size_t)L * hid), s1((size_t)L * inter),
      s2((size_t)L * hid), b1((size_t)L * inter), b2((size_t)L * hid);
  for (int l = 0; l < L; ++l) {
    const std::string p = root + "/layer_" + std::to_string(l);
    RET_IF(read_file(p + "/ln1.bin", buf, (size_t)2 * hid * 4));
    std::memcpy(g1.data() + (size_t)l * hid, buf.data(), hid * 4);
    std::memcpy(be1.data() + (size_t)l * hid, buf.data() + hid * 4, hid * 4);
    RET_IF(read_file(p + "/ln2.bin", buf, (size_t)2 * hid * 4));
    std::memcpy(g2.data() + (size_t)l * hid, buf.data(), hid * 4);
    std::memcpy(be2.data() + (size_t)l * hid, buf.data() + hid * 4, hid * 4);
    struct { const char* name; int8_t* q; float* s; int K, N; } mats[4] = {
        {"attn_wqkv", qqkv.data() + (size_t)l * hid * 3 * hid, sqkv.data() + (size_t)l * 3 * hid, hid, 3 * hid},
        {"attn_wo", qo.data() + (size_t)l * hid * hid, so.data() + (size_t)l * hid, hid, hid},
        {"mlp_fc1", q1.data() + (size_t)l * hid * inter, s1.data() + (size_t)l * inter, hid, inter},
        {"mlp_fc2", q2.data() + (size_t)l * inter * hid, s2.data() + (size_t)l * hid, inter, hid}};
    for (auto& mt : mats) {
      RET_IF(read_file(p + "/" + mt.name + ".i8", buf, (size_t)mt.K * mt.N));
      std::memcpy(mt.q, buf.data(), (size_t)mt.K * mt.N);
      RET_IF(read_file(p + "/" + mt.name + ".scale", buf, (size_t)mt.N * 4));
      std::memcpy(mt.s, buf.data(), (size_t)mt.N * 4);
    }
    RET_IF(read_file(p + "/mlp_biases.bin", buf, (size_t)(inter + hid) * 4));
    std::memcpy(b1.data() + (size_t)l * inter, buf.data(), (size_t)inter * 4);
    std::memcpy(b2.data() + (size_t)l * hid, buf.data() + (size_t)inter * 4, (size_t)hid * 4);
  }
  llm_int8_weights w{emb.data(), g1.data(), be1.data(), g2.data(), be2.data(), qqkv.data(),
                     sqkv.data(), qo.data(), so.data(), q1.data(), s1.data(), b1.data(),
                     q2.data(), s2.data(), b2.data()};
  return llm_decoder_set_int8_weights(d, &w);
}
