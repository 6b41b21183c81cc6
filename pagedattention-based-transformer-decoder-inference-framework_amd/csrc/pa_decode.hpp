// Internal entry of the paged decode attention (csrc/pa_decode.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "llm_decoder.h"

namespace llm {

// pa_decode with a row stride for q (the decoder reads q in place from the
// fused qkv projection output, rows of 3*hid floats).
// Optional per-row conversions of the attention output fused into the split
// merge (the o_proj input): int8 + inv_scale (per-row quantisation) and/or fp16.
struct PaRowOutputs {
  int8_t* q = nullptr;
  float* inv_scale = nullptr;
  void* out16 = nullptr;
  int pack = 0;  // q / out16 in packed-A order (common.hpp a_frag_off_*)
  int keep_out = 1;  // 0: a split launch skips the fp32 `out` rows (only q / out16 are read)
  // 1 (with q and out16 NULL): the consumer quantises the fp32 `out` rows
  // itself (the INT8 o_proj's quantising prologue), so a split launch may
  // merge its splits inside the workgroup and write `out` (no merge launch)
  int f32_rows = 0;
  // FP16 decoder, fused o_proj (workgroup-merge launches only, pa_decode_plan
  // form LLM_PA_FORM_WG_MERGE | LLM_PA_FORM_OPROJ): each (row, head)
  // workgroup multiplies its merged head (rounded to fp16, as the o_proj
  // input) by W_o's rows of that head and adds the o_n products into o_acc
  // row b with atomics (counted fixed point, common.hpp oacc_term; all zero
  // between launches); the adder completing a column writes o_x[b][n] (fp32,
  // what the o_proj GEMM would have written) and clears the column.
  // wo_heads: fp16 [H][D/8][o_n][8] (8 consecutive k of one column per 16 bytes).
  long long* o_acc = nullptr;
  float* o_x = nullptr;
  const void* wo_heads = nullptr;
  int o_n = 0;
  // device int set to 1 when a head's term left the accumulator's range and was
  // clamped (common.hpp oacc_term); required with o_acc
  int* o_flag = nullptr;
  // Beam-group launches (row_group 4, fp16 KV): 2 * ceil(B / 4) * H counters,
  // zero before the first launch and left at zero by every launch; with them
  // the launch assigns tiles dynamically (csrc/tune/pa_beam_steal.hpp,
  // LLM_PA_FORM_STEAL), without them it runs the static BEAM form
  unsigned* beam_ctr = nullptr;
};

// The launch a call takes (pa_decode_plan): splits per (row, head) and
// LLM_PA_FORM_* (| LLM_PA_FORM_BEAM).
struct PaPlan {
  int nsplit = 0;
  int form = 0;
};

// `out` (fp32) may be NULL when `rows` requests an output and the launch splits.
// plan != NULL: only report the launch (q / out / workspace are not needed).
int pa_decode_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                       const int32_t* beam_ids, const int32_t* context_lens, int B, int H, int D,
                       int T, float sm_scale, int pages_per_split, void* workspace,
                       size_t workspace_bytes, hipStream_t st,
                       const PaRowOutputs* rows = nullptr, int row_group = 1,
                       PaPlan* plan = nullptr);
int pa_pages_per_split(int B, int H, int T, int TS, int max_tiles);
// Whether the FP16 decoder fuses its o_proj into the attention's workgroup
// merge (PaRowOutputs::o_acc); always in the product build.
bool oproj_fuse_on();

// Whether the decoder's beam launches assign tiles while they run
// (PaRowOutputs::beam_ctr, csrc/tune/pa_beam_steal.hpp): tuning build, LLM_BEAM_STEAL=1
// (same-box it lost to the static BEAM form).
bool beam_steal_on();

// Split merge of per-(row, head, split) partial softmax states into rows
// (out fp32 [B][H*D] and/or the rows->q / out16 o_proj inputs); row b's
// context is context_lens[b], or ctx_p0 + b + 1 when context_lens is NULL and
// ctx_p0 >= 0, or T.  Split s of a row covers tiles [s*pps, (s+1)*pps).
int pa_merge_rows_internal(const float* part_acc, const float* part_ml, float* out,
                           const PaRowOutputs* rows, const int32_t* context_lens, int ctx_p0,
                           int B, int H, int D, int T, int TS, int pps, int nsplit, int max_tiles,
                           hipStream_t st);

int pa_merge_splits_internal(const float* part_acc, const float* part_ml, float* out,
                             const int32_t* context_lens, int B, int H, int D, int T, int TS,
                             int pps, int nsplit, int max_tiles, hipStream_t st);

// Causal MFMA attention of a prompt chunk (csrc/pa_prefill.hip, C entry
// pa_prefill): out rows i < m = attention of query i (position p0 + i) over
// positions 0 .. p0 + i of page-table row `row`.
// With workspace (pa_prefill_workspace_bytes) the key range is split over
// workgroups and merged by pa_merge_rows_internal, which also writes `rows`
// (the o_proj input); without, one pass writes out and `rows` is converted by
// the row quantiser.  `out` may be NULL only when it splits and rows is set.
bool pa_prefill_supported(const pa_kv_view* kv);
size_t pa_prefill_ws_bytes(const pa_kv_view* kv, int p0, int m);
int pa_prefill_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                        int out_stride, int row, int p0, int m, float sm_scale, void* workspace,
                        size_t workspace_bytes, hipStream_t st, const PaRowOutputs* rows = nullptr);

// Bytes per element of a KV pool type (0: unknown type).
inline int kv_elem_size(int kvt) {
  return kvt == LLM_F16 || kvt == LLM_BF16 ? 2 : kvt == LLM_F32 ? 4 : kvt == LLM_I8 ? 1 : 0;
}

// Bytes from page p to page p + 1 of a view's pools (page_stride 0 = dense).
inline size_t kv_view_page_stride(const pa_kv_view& v) {
  return v.page_stride > 0 ? (size_t)v.page_stride
                           : (size_t)v.page_size * v.head_dim * kv_elem_size(v.kv_dtype);
}

}  // namespace llm
