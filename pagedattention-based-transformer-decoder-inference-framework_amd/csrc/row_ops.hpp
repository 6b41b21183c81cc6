// Internal launchers of csrc/row_ops.hip (used by the decoder runtime).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace llm {

// pack = 1: int8 / fp16 outputs in packed-A order (common.hpp a_frag_off_*;
// needs cols % 64 == 0), consumed by the weight GEMMs with a_packed.
hipError_t launch_quantize_rows(const float* x, int rows, int cols, int8_t* q, float* inv,
                                hipStream_t st, int pack = 0);
struct LnSource;
// pp (optional): read the rows as embedding rows E[tok[r]] instead of x
// (gemm.hpp LnSource)
hipError_t launch_layernorm_quant(const float* x, int rows, int cols, const float* g,
                                  const float* b, float eps, float* out, int8_t* q, float* inv,
                                  hipStream_t st, int pack = 0, const LnSource* pp = nullptr);
hipError_t launch_layernorm_f16(const float* x, int rows, int cols, const float* g,
                                const float* b, float eps, void* out16, hipStream_t st,
                                int pack = 0, const LnSource* pp = nullptr);
hipError_t launch_to_f16(const float* x, size_t n, void* y, hipStream_t st, int pack_cols = 0);
hipError_t launch_advance(int32_t* pos, int32_t* ctx, int n, hipStream_t st);
hipError_t launch_argmax(const float* logits, int rows, int V, int32_t* out, int32_t* out2,
                         int out2_stride, hipStream_t st);
hipError_t launch_embed(const void* E, const int32_t* tok, int rows, int hid, int V, float* x,
                        hipStream_t st);
hipError_t launch_scatter_i32(int32_t* dst, const int64_t* idx, const int32_t* val, int n,
                              hipStream_t st);
// LM head (csrc/lm_head.hip): logits = x . E^T (E packed by launch_lm_pack); with part_val/part_idx also the
// per-(row, workgroup) first maxima that launch_argmax_partials reduces to ids.
int lm_head_workgroups(int V);
size_t lm_head_packed_bytes(int V, int K);
hipError_t launch_lm_pack(const void* E, void* P, int V, int K, hipStream_t st);  // E -> packed
hipError_t launch_lm_head(const float* x, const void* E, float* logits, int M, int V, int K,
                          float* part_val, int32_t* part_idx, hipStream_t st);
hipError_t launch_argmax_partials(const float* part_val, const int32_t* part_idx, int M, int nwg,
                                  int32_t* out, hipStream_t st, int32_t* pos = nullptr,
                                  int32_t* ctx = nullptr);
// Device sampling (csrc/sample.hip); counter[r] is the per-row draw counter.
hipError_t launch_sample(const float* logits, int rows, int row0, int V, float temperature,
                         int top_k, float top_p, uint64_t seed, const int32_t* counter,
                         int32_t* out, hipStream_t st);
// Seeded uniform (variance-1 x scale) fp16 over `pages` pages of page_elems
// elements, page p at p + p * page_stride elements.
hipError_t launch_fill_random_f16(void* p, size_t pages, size_t page_elems, size_t page_stride,
                                  uint64_t seed, float scale, hipStream_t st);

}  // namespace llm
