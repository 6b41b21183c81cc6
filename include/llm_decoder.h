/*
 * llm_decoder.h — C ABI of the MI355X (gfx950) paged-attention decode path.
 *
 * This is the drop-in boundary: plain pointers, sizes and opaque handles, no
 * torch or HIP types (a hipStream_t is passed as `void*`).  Every entry point
 * returns 0 (LLM_OK) or one of the llm_status codes; llm_last_error() gives a
 * message for the calling thread.  The pybind11 module `llm_decoder`
 * (csrc/bindings.cpp) wraps these exactly as the reference's
 * src/bindings.cpp:3-35 exposes its classes, mapping non-zero status to
 * RuntimeError (the reference's loaders throw std::runtime_error,
 * decoder/decoder_block.hpp:13-19).
 *
 * Citations are file:line in the reference tree.
 */
#ifndef LLM_DECODER_H_
#define LLM_DECODER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum llm_status {
  LLM_OK = 0,
  LLM_ERR_INVALID = 1,      /* bad shape / argument (checked on the host before any launch) */
  LLM_ERR_UNSUPPORTED = 2,  /* valid request this build does not implement (e.g. top-k in attention) */
  LLM_ERR_HIP = 3,          /* HIP runtime error */
  LLM_ERR_OOM = 4,          /* device or page-pool allocation failure */
  LLM_ERR_IO = 5,           /* weight / cache file I/O */
  LLM_ERR_RANGE = 6         /* a device value left a fixed-point accumulator's range (the
                               FP16 decoder's fused o_proj); reported ONCE per clamp, by the
                               first llm_decoder_sync or synchronous step after it */
};

/* Element types.  KV pools may be any of the four (the T of
 * AttentionCUDA::forward, attention/attention_cuda.cu:58-94: __half, bf16,
 * int8_t (raw values, no scale), float); weights are LLM_I8 or LLM_F16. */
enum llm_dtype { LLM_F16 = 0, LLM_I8 = 1, LLM_F32 = 2, LLM_BF16 = 3 };
enum llm_act { LLM_ACT_NONE = 0, LLM_ACT_RELU = 1, LLM_ACT_GELU = 2 };

const char* llm_last_error(void);
int llm_abi_version(void);

/* ------------------------------------------------------------------------ */
/* Paged decode attention                                                    */
/* ------------------------------------------------------------------------ */

/* POD device view of one layer's KV pools + page table, passed BY VALUE to the
 * kernel.  Replaces handing the host KVTileCache object (std containers,
 * mutex) to device code (attention/attention_tile_launcher.hpp:43,
 * attention/paged_flash_attention_kernel_fused.cu:13).  Semantics of
 * KVTileCache<T>::get (kv_cache/kv_tile_cache.hpp:21-26) and
 * PageTable::lookup (kv_cache/page_table.hpp:39-49): entry
 * page_table[(beam*num_heads + head)*max_tiles + tile]; a page < 0 or
 * >= num_pages means "no tile" (its tokens are masked). */
typedef struct pa_kv_view {
  const void* k_pool;         /* [num_pages][page_size][head_dim] of kv_dtype */
  const void* v_pool;         /* same layout */
  const int32_t* page_table;  /* [num_beams][num_heads][max_tiles] int32, device */
  int32_t num_pages;
  int32_t page_size;          /* tokens per page (tile_size) */
  int32_t head_dim;
  int32_t num_beams;
  int32_t num_heads;
  int32_t max_tiles;
  int32_t kv_dtype;           /* LLM_F16 (default), LLM_BF16, LLM_F32 or LLM_I8; one page
                               * (page_size * head_dim elements) must be 1..16 KiB */
  int64_t page_stride;        /* bytes from page p to page p + 1 within each pool; 0 = one
                               * page (dense pools).  kv_cache's own pools interleave K and
                               * V pages ([num_pages][K page | V page], stride 2 pages,
                               * v_pool = k_pool + 1 page) */
} pa_kv_view;

/* Bytes of device workspace pa_decode needs (split-T partial softmax state). */
size_t pa_decode_workspace_bytes(int B, int H, int D, int max_tiles, int pages_per_split);

/* Host-only ESTIMATE of the split-T size pa_decode picks when
 * pages_per_split <= 0, for a uniform context T: it assumes 3,072 resident
 * waves (256 CUs x 12) where pa_decode queries the device's occupancy for the
 * kernel it launches and derives each row's split length from that row's own
 * context, so the two can differ.  For labelling runs, not for sizing them. */
int pa_decode_pages_per_split(int B, int H, int T, int page_size, int max_tiles);

/* The launch a pa_decode / pa_decode_grouped call with these arguments
 * takes, without launching it: *nsplit = splits per (row, head) and *form =
 * LLM_PA_FORM_* (direct: one split, no merge; split + merge launch;
 * LLM_PA_FORM_BEAM is or-ed in for the beam-group kernel).  For tests and
 * run labels; the decoder's own step reports its launch with
 * llm_decoder_attention_plan. */
#define LLM_PA_FORM_DIRECT 0
#define LLM_PA_FORM_SPLIT_MERGE 1     /* split launch + pa_merge_kernel (fp32 rows) */
#define LLM_PA_FORM_SPLIT_MERGE_ROW 2 /* split launch + pa_merge_row_kernel (o_proj input) */
#define LLM_PA_FORM_WG_MERGE 3        /* splits merged inside the split workgroup */
#define LLM_PA_FORM_BEAM 16
#define LLM_PA_FORM_OPROJ 32 /* FP16 decoder: o_proj fused into the workgroup merge */
#define LLM_PA_FORM_STEAL 64 /* tuning library only (LLM_BEAM_STEAL=1): beam groups with
                                tiles assigned to the splits while the launch runs (with
                                LLM_PA_FORM_BEAM); the product never reports it */
int pa_decode_plan(const pa_kv_view* kv, int B, int H, int D, int T, int pages_per_split,
                   int row_group, int* nsplit, int* form);

/* Paged decode attention (replaces paged_flash_attention_kernel_fused,
 * attention/paged_flash_attention_kernel_fused.cu:5-90, launched by
 * AttentionTileLauncher::launch, attention/attention_tile_launcher.hpp:36-89,
 * from AttentionCUDA::forward, attention/attention_cuda.cu:41-95), with the
 * INTENDED maths of cpu_paged_attention_forward
 * (attention_cpu/cpu_attention_kernel.cpp:37-129):
 *   r = beam_ids ? beam_ids[b] : b;  T_b = context_lens ? context_lens[b] : T
 *   s_t = (q[b,h] . k_t) * sm_scale        (sm_scale = 1/temperature^2 reproduces
 *                                           the reference's double division)
 *   out[b,h] = sum_t exp(s_t - max s) v_t / (sum_t exp(s_t - max s) + 1e-6)
 * over t < T_b whose page is present.  q, out: fp32 [B][H][D] device.
 * pages_per_split <= 0: the split count is chosen on the device side of the
 * call from the launch's occupancy (a whole number of resident-wave rounds)
 * and each row's split length from its own context; pa_decode_pages_per_split
 * only estimates it, and pa_decode_plan reports the choice exactly.
 * workspace may be NULL when the call needs none (single split). */
int pa_decode(const pa_kv_view* kv, const float* q, float* out, const int32_t* beam_ids,
              const int32_t* context_lens, int B, int H, int D, int T, float sm_scale,
              int pages_per_split, void* workspace, size_t workspace_bytes, void* stream);

/* pa_decode with beam-aware scheduling (the beam routing of
 * paged_flash_attention_kernel_fused.cu:22 plus "beam-aware KV tile prefetch",
 * README.md:64): rows are taken in groups of row_group (1..4, e.g. the beams of
 * one sequence, rows g*row_group .. g*row_group+row_group-1); the group's rows
 * for one (head, split) run as adjacent waves of one workgroup, so KV pages
 * they share through kv_cache_fork are read from HBM once (row_group 4: staged
 * through LDS, with split boundaries placed by cost so the splits holding the
 * beam-private tail are not the slowest).  Results equal pa_decode bit for
 * bit, except for groups of 4 equal-context rows under dynamic splits
 * (pages_per_split 0), whose cost-balanced partition changes only the fp32
 * rounding of the split merge.  The workspace is sized by
 * pa_decode_workspace_bytes as for pa_decode. */
int pa_decode_grouped(const pa_kv_view* kv, const float* q, float* out, const int32_t* beam_ids,
                      const int32_t* context_lens, int B, int H, int D, int T, float sm_scale,
                      int pages_per_split, int row_group, void* workspace,
                      size_t workspace_bytes, void* stream);

/* Causal paged attention of a prompt chunk: the reference's prefill pass
 * (AttentionCUDA's is_prefill flag, attention/attention_cuda.hpp:21; maths of
 * cpu_paged_attention_forward, attention_cpu/cpu_attention_kernel.cpp:37-129,
 * per query).  m query tokens of ONE sequence at positions p0 .. p0+m-1, whose
 * K/V are already in the pages of page-table row `row`; query i attends to
 * positions 0 .. p0+i.  Equals pa_decode with B = m, beam_ids[i] = row,
 * context_lens[i] = p0 + i + 1 (within 1e-3 relative), but each K/V page is
 * read once per 32 queries instead of once per query (MFMA tiles).
 * q, out: fp32 [m][H][D] with row strides q_stride / out_stride floats
 * (<= 0: H*D), 16-byte aligned.  fp16 pools, head_dim 64 or 128, page_size
 * 16 or 32 (else LLM_ERR_UNSUPPORTED; pa_decode covers every shape).
 * With workspace_bytes >= pa_prefill_workspace_bytes(kv, p0, m) (and
 * out_stride H*D) the key range is split over more workgroups and merged as
 * pa_decode's splits; with less (or NULL) it runs in one pass. */
size_t pa_prefill_workspace_bytes(const pa_kv_view* kv, int p0, int m);
int pa_prefill(const pa_kv_view* kv, const float* q, int q_stride, float* out, int out_stride,
               int row, int p0, int m, float sm_scale, void* workspace, size_t workspace_bytes,
               void* stream);

/* The optional stages of the reference attention, CPUAttentionInput /
 * CPUAttentionOutput (attention_cpu/attention_cpu.hpp:8-43) as used by
 * cpu_paged_attention_forward (attention_cpu/cpu_attention_kernel.cpp:37-129):
 *   scores_t = q.k_t / temperature (-1e9 where the tile is missing)
 *   p = exp((scores - max) / temperature) / (sum + 1e-6)  (softmax_lut.cpp:203-231)
 *   apply_topk_topp_filter (softmax_lut.cpp:233-256): rank by (p, index)
 *     descending, zero rank >= top_k (top_k > 0) and every entry whose
 *     higher-ranked mass is >= top_p (top_p < 1); no renormalisation; then if
 *     eos_token >= 0 and p[eos_token] > eos_threshold, zero all other entries
 *   out = sum_t p_t v_t
 * The GPU kernel of the reference exposes the same knobs (top_k, top_p,
 * rerank_scores: paged_flash_attention_kernel_fused.cu:5-90). */
typedef struct pa_decode_options {
  float temperature;   /* > 0; 1 = reference default (attention_config.hpp:20) */
  int top_k;           /* 0 = off */
  float top_p;         /* 1 = off */
  int eos_token;       /* -1 = off (a KV position) */
  float eos_threshold;
  float* probs_out;    /* [B][H][T] attention weights after filtering, 0 past T_b (nullable) */
  float* scores_out;   /* [B][H][T] scores, -1e9 past T_b / for missing tiles (nullable) */
} pa_decode_options;

/* pa_decode with the options above.  With every option off (top_k 0, top_p 1,
 * eos -1, no outputs) this is pa_decode with sm_scale = 1/temperature^2 (the
 * hot path; workspace as for pa_decode).  Otherwise one workgroup per (b, h)
 * keeps the row's scores in LDS when T <= 8192 (workspace unused), and in the
 * workspace for longer rows: T > 8192 needs an 8-byte aligned workspace of
 * pa_decode_ex_workspace_bytes(B, H, T) bytes (else LLM_ERR_INVALID); like
 * cpu_paged_attention_forward (attention_cpu/cpu_attention_kernel.cpp:61) the
 * context has no practical upper bound: D <= 256 and T <= 2^30 (else
 * LLM_ERR_UNSUPPORTED; the workspace size is then 0). */
size_t pa_decode_ex_workspace_bytes(int B, int H, int T);
int pa_decode_ex(const pa_kv_view* kv, const float* q, float* out, const int32_t* beam_ids,
                 const int32_t* context_lens, int B, int H, int D, int T,
                 const pa_decode_options* opt, void* workspace, size_t workspace_bytes,
                 void* stream);

/* ------------------------------------------------------------------------ */
/* INT8 / FP16 weight GEMMs (MFMA)                                          */
/* ------------------------------------------------------------------------ */

/* Bytes of the packed (MFMA-fragment-ordered) weight for a [K][N] matrix. */
size_t gemm_packed_bytes(int dtype, int K, int N);

/* Repack W [K][N] row-major (the reference layout, decoder/mlp.hpp:28-31) into
 * the MFMA fragment order the GEMM streams (device -> device). */
int gemm_pack_weights(int dtype, const void* W_kn, void* W_packed, int K, int N, void* stream);

/* INT8 GEMM, contract of dnnl_matmul_int8 (attention_cpu/dnnl_matmul_int8.cpp:7-75)
 * restated for decode:
 *   acc[m,n] = sum_k int32(A[m,k]) * int32(W[k,n])          exact int32
 *   C[m,n]   = act(float(acc) * (sa[m] * sw[n]) + bias[n])  fp32
 * A int8 [M][K] (row stride lda >= K), W_packed from gemm_pack_weights.
 * sa / sw / bias may be NULL (1, 1, 0).  acc_out (int32 [M][N]) and C
 * (fp32 [M][N]) may each be NULL.  K % 64 == 0, N % 16 == 0. */
int i8_gemm(const int8_t* A, int lda, const void* W_packed, int32_t* acc_out, float* C,
            int M, int N, int K, const float* sa, const float* sw, const float* bias,
            int act, void* stream);

/* Batched INT8 matmul with int8 output, the full form of dnnl_matmul_int8
 * (attention_cpu/dnnl_matmul_int8.cpp:7-75, dnnl_matmul_int8.hpp:5-13):
 *   A s8 [batch][M][K], B s8 [batch][K][N] (row-major, unpacked), C s8 [batch][M][N]
 *   y = act((float(acc) + bias[n]) * alpha),  alpha = scale_a * scale_b / scale_c
 *   C = round_half_even(saturate(y, -128, 127))
 * bias (fp32 [N]) may be NULL; act LLM_ACT_NONE / RELU / GELU (erf).  Any M, N,
 * K (K < 131072); batch * M * N == 0 is a no-op.  The reference returns false
 * on any failure; this returns a status code (llm_last_error()). */
int i8_matmul_s8(const int8_t* A, const int8_t* B, int8_t* C, int batch, int M, int N, int K,
                 float scale_a, float scale_b, float scale_c, const float* bias, int act,
                 void* stream);

/* FP16 GEMM with fp32 accumulate (CUDADecoder weights):
 *   C[m,n] = act(sum_k A[m,k] W[k,n] + bias[n]),  A fp16 [M][K], K % 32 == 0. */
int f16_gemm(const void* A, int lda, const void* W_packed, float* C, int M, int N, int K,
             const float* bias, int act, void* stream);

/* Tied-embedding LM head: logits[m,v] = sum_k x[m,k] * E[v,k], x fp32 [M][K],
 * E fp16 [V][K] (token_embedding.hpp layout).  x is split hi+lo into two fp16
 * MFMA operands so the product keeps ~fp32 accuracy.  K % 32 == 0. */
int lm_head(const float* x, const void* E, float* logits, int M, int V, int K, void* stream);

/* Row-wise argmax (first maximum wins, std::max_element, decoder/cuda_decoder.cu:7-14). */
int argmax_rows(const float* logits, int rows, int V, int32_t* out, void* stream);

/* Device token sampling per row, reference semantics of
 * top_k_top_p_filter (attention/top_k_top_p_filter.cuh:55-111) and
 * apply_topk_topp_filter (attention_cpu/softmax_lut.cpp:233-256):
 *   p = softmax(logits / temperature) (max-subtracted, sum + 1e-6);
 *   token i is dropped if its probability rank >= top_k (top_k > 0) or if the
 *   probability mass ranked above it is >= top_p (top_p < 1);
 *   the kept mass is sampled by inverse CDF in token-index order with
 *   u = sample_uniform_host(seed, row, counter) in [0, 1).
 * temperature <= 0 or top_k == 1: greedy argmax (cuda_decoder.cu:7-14).
 * V <= 65536. */
int sample_rows(const float* logits, int rows, int V, float temperature, int top_k, float top_p,
                uint64_t seed, int counter, int32_t* out, void* stream);
/* The uniform draw sample_rows uses for (seed, row, counter): splitmix64 of
 * seed ^ (row << 32) ^ counter, top 24 bits / 2^24. */
float sample_uniform_host(uint64_t seed, int row, int counter);

/* Per-row dynamic int8 quantisation (attention_cpu/int8_quant.cpp:5-13,59-64):
 * scale_r = 127/(absmax_r + 1e-6); q = clamp(round(x*scale_r)); inv_scale[r] = 1/scale_r. */
int quantize_rows(const float* x, int rows, int cols, int8_t* q, float* inv_scale, void* stream);

/* LayerNorm (decoder/layer_norm.hpp:20-37) fused with per-row int8 quantisation
 * (q/inv_scale may be NULL: then only `out` fp32 is written; out may be NULL). */
int layernorm_quant(const float* x, int rows, int cols, const float* gamma, const float* beta,
                    float eps, float* out, int8_t* q, float* inv_scale, void* stream);

/* ------------------------------------------------------------------------ */
/* KV cache: page pools + page table (kv_cache/page_table.hpp:5-37,          */
/* kv_cache/kv_tile_cache.hpp:9-80) with a layer dimension, a free-list page */
/* allocator (replacing the map.size() ids of kv_tile_cache.cpp:71) and a    */
/* single host source of truth synchronised to the device.                   */
/* ------------------------------------------------------------------------ */
typedef struct kv_cache kv_cache;

int kv_cache_create(int num_layers, int num_beams, int num_heads, int head_dim, int page_size,
                    int max_tiles, long long num_pages, kv_cache** out);
/* kv_cache_create with pools of kv_dtype elements (KVTileCache<T>,
 * kv_cache/kv_tile_cache.hpp:9 with T in {__half, bf16, int8_t, float}). */
int kv_cache_create_typed(int num_layers, int num_beams, int num_heads, int head_dim,
                          int page_size, int max_tiles, long long num_pages, int kv_dtype,
                          kv_cache** out);
void kv_cache_destroy(kv_cache* c);
int kv_cache_view(const kv_cache* c, int layer, pa_kv_view* out);
long long kv_cache_num_pages(const kv_cache* c);
long long kv_cache_free_pages(const kv_cache* c);
/* PageTable::assign (page_table.cpp:49-53) / lookup / remove (:64-66), host mirror. */
int kv_cache_assign(kv_cache* c, int layer, int beam, int head, int tile, int page);
int kv_cache_lookup(const kv_cache* c, int layer, int beam, int head, int tile);
int kv_cache_remove(kv_cache* c, int layer, int beam, int head, int tile);
/* KVTileCache::register_tile (kv_tile_cache.cpp:64-77): allocate a free page
 * for (layer, beam, head, tile) if it has none; returns the page id in *page. */
int kv_cache_register_tile(kv_cache* c, int layer, int beam, int head, int tile, int* page);
/* Page-pool exhaustion policy of kv_cache_register_tile.  LLM_EVICT_NONE (the
 * default): LLM_ERR_OOM.  LLM_EVICT_LRU: KVTileCache's policy
 * (kv_cache/kv_tile_cache.cpp:64-98, update_lru / evict_if_needed): every
 * register_tile call makes its tile the most recently used, and a tile that
 * needs a page when none is free takes one by removing the least recently
 * registered tile whose page that frees (an entry on a page a forked beam
 * still shares is kept) -- the reference's semantics, so an evicted tile of a
 * live sequence reads as missing (masked) afterwards.  Only entries whose
 * page kv_cache_register_tile mapped are candidates: any other call that
 * writes an entry (reserve / the decoder's append, assign -- even with its
 * current page --, remove, release, fork, copy-on-write, a snapshot load)
 * takes it off the recency list, so the decoder's own pages never are.
 * Switching the policy keeps the recency list. */
#define LLM_EVICT_NONE 0
#define LLM_EVICT_LRU 1
int kv_cache_set_eviction(kv_cache* c, int policy);
/* Ensure pages exist for tiles covering tokens [0, n_tokens) of `beam`, all layers/heads. */
int kv_cache_reserve(kv_cache* c, int beam, int n_tokens);
/* Beam fork: dst's page-table rows := src's (all layers, heads), shared pages
 * refcounted; pages of dst are copied-on-write by kv_cache_append/write. */
int kv_cache_fork(kv_cache* c, int src_beam, int dst_beam);
/* Release every page of `beam` (refcount-aware). */
int kv_cache_release(kv_cache* c, int beam);
/* PageTable::clear (page_table.cpp:39-44): all entries -1, all pages free. */
int kv_cache_clear(kv_cache* c);
/* PageTable::sync_to_gpu (page_table.cpp:59-62): push dirty host entries. */
int kv_cache_sync(kv_cache* c, void* stream);
/* Copy n tokens of K and V (host, [n][H][D] in the cache's kv_dtype) for
 * `beam` starting at token position pos into the pools of `layer`. */
int kv_cache_write_tokens(kv_cache* c, int layer, int beam, int pos, int n, const void* k_host,
                          const void* v_host);
/* Device pointers of the pools / table (for tests and custom kernels).  Page
 * p of the K (V) pool starts at kv_cache_k_pool (v_pool) + p * page_stride. */
void* kv_cache_k_pool(kv_cache* c);
void* kv_cache_v_pool(kv_cache* c);
long long kv_cache_page_stride(const kv_cache* c);
int32_t* kv_cache_page_table(kv_cache* c, int layer);
/* Snapshot of the whole cache ("APPIMKV2": geometry, layered page table, used
 * pages K then V) — this build's own format, the one that restores the page
 * table too.  kv_cache_load validates the whole file (geometry, every table
 * entry and page id in [-1, num_pages), exact size) before it changes the
 * cache; on a failure after that point the cache is left cleared. */
int kv_cache_save(const kv_cache* c, const char* path);
int kv_cache_load(kv_cache* c, const char* path);
/* Validate a snapshot on the host (no device needed): geometry[9] receives
 * {L, beams, H, D, page_size, max_tiles, num_pages, kv_dtype, used_pages}. */
int kv_cache_inspect(const char* path, long long* geometry);
/* KVTileCache<T>::save_to_file / load_from_file (kv_cache/kv_tile_cache.cpp:
 * 105-125), byte for byte: the raw K pool [num_pages][page_size][head_dim]
 * then the raw V pool, no header, no page table (the reader keeps its own).
 * load_pools refuses a file whose size is not 2 * num_pages * page bytes. */
int kv_cache_save_pools(const kv_cache* c, const char* path);
int kv_cache_load_pools(kv_cache* c, const char* path);
/* KVTileCacheCPU<T>::save / load (kv_cache/kv_tile_cache_cpu.cpp:89-123), byte
 * for byte: int32 count, then per tile {int32 batch_id, head_id, tile_id} and
 * page_size * head_dim elements.  One file holds the K (kind 0) or V (kind 1)
 * tiles of one layer (the reference keeps K and V in two caches); batch_id is
 * the beam.  save writes every mapped tile in (beam, head, tile) order (the
 * reference's order is its hash map's).  load maps each record's tile (a new
 * page, or copy-on-write of a shared one) and writes its data; a later record
 * of the same tile wins, as in the reference; records outside this cache's
 * (beam, head, tile) range are refused before anything changes. */
int kv_cache_save_tiles(const kv_cache* c, int layer, int kind, const char* path);
int kv_cache_load_tiles(kv_cache* c, int layer, int kind, const char* path);
/* Validate a tile-record file of tile_bytes-byte tiles on the host (no device
 * needed); *count receives its record count. */
int kv_tiles_inspect(const char* path, long long tile_bytes, int* count);

/* ------------------------------------------------------------------------ */
/* Decoder (CUDADecoder / INT8Decoder, decoder/cuda_decoder.hpp:7-21,        */
/* decoder/int8_decoder.hpp:6-17)                                            */
/* ------------------------------------------------------------------------ */
typedef struct llm_decoder llm_decoder;

typedef struct llm_decoder_config {
  int num_layers, num_heads, head_dim, hidden_dim, vocab_size, max_seq_len; /* ctor args, bindings.cpp:6 */
  int inter_dim;        /* 0 -> 4*hidden_dim (decoder_block.hpp:28) */
  int page_size;        /* 0 -> 16 */
  int weight_dtype;     /* LLM_I8 (INT8Decoder) or LLM_F16 (CUDADecoder) */
  int max_batch;        /* rows decoded together (0 -> 1) */
  float attn_scale;     /* score multiplier; 1.0 = reference (no 1/sqrt(D)) */
  long long num_pages;  /* KV page-pool size; 0 -> enough for max_batch * max_seq_len */
} llm_decoder_config;

int llm_decoder_create(const llm_decoder_config* cfg, llm_decoder** out);
void llm_decoder_destroy(llm_decoder* d);

/* Host weights (row-major reference layouts), uploaded and packed on device.
 * INT8: wqkv [L][hid][3hid] (q|k|v, heads contiguous), wo [L][hid][hid],
 * w1 [L][hid][inter], w2 [L][inter][hid] int8 + per-output-column fp32 dequant
 * scales; biases b1 [L][inter], b2 [L][hid]; LayerNorm gamma/beta [L][hid];
 * emb fp16 [V][hid] (embedding and tied LM head). */
typedef struct llm_int8_weights {
  const uint16_t* emb;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  const int8_t* wqkv; const float* sw_qkv;
  const int8_t* wo;   const float* sw_o;
  const int8_t* w1;   const float* sw1; const float* b1;
  const int8_t* w2;   const float* sw2; const float* b2;
} llm_int8_weights;
int llm_decoder_set_int8_weights(llm_decoder* d, const llm_int8_weights* w);

typedef struct llm_f16_weights {
  const uint16_t* emb;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  const uint16_t *wqkv, *wo, *w1, *w2;   /* fp16, same [K][N] layouts */
  const float *b1, *b2;
} llm_f16_weights;
int llm_decoder_set_f16_weights(llm_decoder* d, const llm_f16_weights* w);

/* CUDADecoder::load_weights (decoder/cuda_decoder.cu:35-45) / INT8Decoder::
 * load_quantized_weights (decoder/int8_decoder.cpp:91-95) / quantize_weights
 * (:43-89) over the raw little-endian .bin layout of weights/README.md:26-38. */
int llm_decoder_load_weights(llm_decoder* d, const char* dir);
int llm_decoder_load_quantized_weights(llm_decoder* d, const char* dir);
int llm_quantize_weights(const char* fp32_dir, const char* int8_dir, int num_layers,
                         int hidden_dim, int inter_dim, int vocab_size);

/* Batched generate (CUDADecoder<T>::generate, decoder/cuda_decoder.cu:48-61,
 * batched): for each row, prompt tokens are consumed one per step (KV is
 * appended), then max_gen_len tokens are produced by greedy argmax.  out
 * [batch][max_gen_len] receives the generated ids (prompt excluded).  A step
 * whose fused o_proj clamped does not stop generation: `out` is filled to the
 * end and LLM_ERR_RANGE is returned afterwards. */
int llm_decoder_generate(llm_decoder* d, const int32_t* prompts, const int32_t* prompt_lens,
                         int prompt_stride, int batch, int max_gen_len, float temperature,
                         int32_t* out);

/* Chunked prefill (the is_prefill pass of AttentionCUDA::forward,
 * attention/attention_cuda.hpp:21): append the n tokens (host ids) of active
 * row `row` at its next positions in one layer pass per chunk of <= 512 tokens
 * (M = chunk weight GEMMs; causal paged attention per token), then set the
 * row's next token from the last token's logits, so llm_decoder_step(tokens =
 * NULL) continues decoding.  llm_decoder_generate uses it for every prompt. */
int llm_decoder_prefill(llm_decoder* d, int row, const int32_t* tokens, int n);

/* Token choice of every following step: greedy argmax (temperature <= 0 or
 * top_k == 1; the default, sample_from_logits, decoder/cuda_decoder.cu:7-14)
 * or device sampling with temperature / top_k / top_p (sample_rows; the draw
 * counter of a row is its position, so runs are replayable for a seed). */
int llm_decoder_set_sampling(llm_decoder* d, float temperature, int top_k, float top_p,
                             uint64_t seed);

/* Low-level stepping (bench / multi-GPU driver). */
/* Start `batch` rows whose first context_len tokens are synthetic: every page
 * is allocated (shuffled order when shuffle != 0) and filled with seeded
 * random fp16 K/V on device. */
int llm_decoder_begin_synthetic(llm_decoder* d, int batch, int context_len, uint64_t seed,
                                int shuffle);
/* Start num_seqs * beam_width rows (row = seq * beam_width + beam) for beam
 * decode: each sequence's first shared_len tokens live in beam 0's pages and
 * are shared by the other beams through kv_cache_fork (refcounted, copy-on-
 * write on append); every beam then holds beam_len private tokens.  Pages hold
 * seeded random fp16 K/V.  Attention runs beam-aware (pa_decode_grouped with
 * row_group = beam_width, 1..4). */
int llm_decoder_begin_beams(llm_decoder* d, int num_seqs, int beam_width, int shared_len,
                            int beam_len, uint64_t seed, int shuffle);
/* One decode step for all active rows: tokens (host [batch], or NULL to feed
 * back the previous argmax) at each row's next position; writes fp32 logits
 * to logits_dev ([batch][V] device, may be NULL) and copies next ids to
 * next_host (may be NULL; a NULL next_host keeps the step asynchronous).
 * stream NULL -> the decoder's own stream. */
int llm_decoder_step(llm_decoder* d, const int32_t* tokens, float* logits_dev,
                     int32_t* next_host, void* stream);
/* Wait for the device.  LLM_ERR_RANGE if, since the last report, a step's
 * fused o_proj (FP16 decoders, LLM_PA_FORM_OPROJ) met a head product outside
 * its fixed-point range ((2^23 - 1) / num_heads in magnitude, or not finite):
 * that product was clamped, so the affected x values are wrong, but the
 * accumulator columns stayed consistent and later steps are unaffected by it.
 * A step with next_host reports the same.  Each clamp is reported once: the
 * report clears the device flag, so later steps and syncs succeed unless they
 * clamp again.  llm_decoder_run_attention launches carry a flag of their own
 * and never make a step or a sync fail. */
int llm_decoder_sync(llm_decoder* d);
/* Health of the fused o_proj after waiting for the device: *clamped = 1 if a
 * step's term was clamped since the last begin / generate, reported or not
 * (see llm_decoder_sync),
 * *nonzero_columns = accumulator columns not back at zero (0 between steps
 * unless a launch was interrupted).  Either pointer may be NULL.  Decoders
 * without the fused o_proj report 0 / 0. */
int llm_decoder_oproj_status(llm_decoder* d, int* clamped, long long* nonzero_columns);
/* Enqueue on `stream` (NULL: the decoder's) a device copy of the last step's
 * next ids (int32 [batch], the greedy argmax or the sampled ids) to dst_dev:
 * the ids-only gather of the multi-GPU path without a host sync. */
int llm_decoder_copy_next(llm_decoder* d, int32_t* dst_dev, void* stream);
/* Activation taps for parity checks: every following
 * llm_decoder_step also copies, per layer l and stage s (0: LN1 output, 1:
 * attention output, 2: LN2 output, 3: fc1 output -- the four int8 GEMM inputs
 * of DecoderBlock::forward, decoder/decoder_block.hpp:43-61), the rows' int8
 * activations in packed-A order (common.hpp a_frag_off_i8) to
 *   q_dev + ((l*4 + s) * ceil(max_batch/16)*16 + row) * K   (K = hidden_dim, or
 *                                                           inter_dim at s = 3;
 *   slot stride ceil(max_batch/16)*16 * max(hidden_dim, inter_dim) bytes)
 * and their fp32 dequantisation scales to s_dev[(l*4 + s) * max_batch + row].
 * FP16 decoders (CUDADecoder) tap their four fp16 GEMM inputs in packed-A
 * order (a_frag_off_f16), at the same slot layout with 2 bytes per element;
 * s_dev is not written (give any device buffer).
 * Both NULL switches the taps off.  Prefill chunks are not tapped. */
int llm_decoder_set_taps(llm_decoder* d, int8_t* q_dev, float* s_dev);
/* The attention launch of the decoder's step at its current batch and row
 * group (pa_decode_plan of layer 0's view, T = max_seq_len: the step graph's
 * launch, whose split lengths follow each row's live context).  INT8 decoders
 * whose o_proj quantises its own input (decode rows <= 64, hidden <= 2048, no
 * beam groups) report the fp32-row forms (LLM_PA_FORM_WG_MERGE up to 8
 * splits, else LLM_PA_FORM_SPLIT_MERGE, LLM_PA_FORM_DIRECT); wider models
 * LLM_PA_FORM_WG_MERGE when their fp32-row plan is one (a quantise launch
 * follows it), else LLM_PA_FORM_SPLIT_MERGE_ROW; beam groups
 * LLM_PA_FORM_SPLIT_MERGE_ROW | LLM_PA_FORM_BEAM.  FP16
 * decoders whose launch merges in the workgroup (2..8 splits, head_dim <= 128,
 * <= 64 heads) run o_proj inside it: LLM_PA_FORM_WG_MERGE | LLM_PA_FORM_OPROJ. */
int llm_decoder_attention_plan(llm_decoder* d, int* nsplit, int* form);
/* Enqueue layer `layer`'s attention launch of the decoder's step on `stream`
 * (NULL: the decoder's) -- the same kernels, grid and outputs as inside the
 * step graph (q from the last step's projection, each row's live context, the
 * o_proj input written), for timing the step's own launch in isolation.  The
 * fused o_proj of an FP16 decoder accumulates into a scratch set of columns of
 * its own here (not the step's), so a run may overlap an in-flight step; two
 * runs of one decoder must not overlap each other. */
int llm_decoder_run_attention(llm_decoder* d, int layer, void* stream);
int llm_decoder_context_len(const llm_decoder* d, int row);
kv_cache* llm_decoder_kv(llm_decoder* d);

#ifdef __cplusplus
}
#endif

#endif /* LLM_DECODER_H_ */
