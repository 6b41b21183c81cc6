// Internal entry of the paged decode attention (csrc/pa_decode.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "llm_decoder.h"

namespace llm {

// pa_decode with a row stride for q (the decoder reads q in place from the
// fused qkv projection output, rows of 3*hid floats).
int pa_decode_internal(const pa_kv_view* kv, const float* q, int q_stride, float* out,
                       const int32_t* beam_ids, const int32_t* context_lens, int B, int H, int D,
                       int T, float sm_scale, int pages_per_split, void* workspace,
                       size_t workspace_bytes, hipStream_t st);
int pa_pages_per_split(int B, int H, int T, int TS, int max_tiles);

}  // namespace llm
