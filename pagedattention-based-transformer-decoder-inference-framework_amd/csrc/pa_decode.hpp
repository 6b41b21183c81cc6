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
};

// `out` (fp32) may be NULL when `rows` requests an output and the launch splits.
int pa_decode_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                       const int32_t* beam_ids, const int32_t* context_lens, int B, int H, int D,
                       int T, float sm_scale, int pages_per_split, void* workspace,
                       size_t workspace_bytes, hipStream_t st,
                       const PaRowOutputs* rows = nullptr, int row_group = 1,
                       int waves_per_simd = 0);
int pa_pages_per_split(int B, int H, int T, int TS, int max_tiles);

// Causal MFMA attention of a prompt chunk (csrc/pa_prefill.hip, C entry
// pa_prefill): out rows i < m = attention of query i (position p0 + i) over
// positions 0 .. p0 + i of page-table row `row`.
bool pa_prefill_supported(const pa_kv_view* kv);
int pa_prefill_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                        int out_stride, int row, int p0, int m, float sm_scale, hipStream_t st);

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
