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

}  // namespace llm
