// Internal entries of csrc/gemm.hip used by the decoder runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "llm_decoder.h"

namespace llm {

// Where the fused qkv projection writes K and V: the pages of position pos[m]
// of row m (page_table already offset to the first row of the launch).
struct KvAppendView {
  const int32_t* pos;
  const int32_t* page_table;
  const int32_t* rows;  // page-table row of GEMM row m (NULL: row m)
  void* k_pool;
  void* v_pool;
  int num_beams = 0, max_tiles = 0, page_size = 0, num_pages = 0, H = 0, D = 0;
  size_t page_stride = 0;  // fp16 elements from page p to page p + 1 (0: one page)
};

// One decode weight GEMM (decoder-internal form of i8_gemm / f16_gemm):
//   C[m, n] = act(acc[m, n] * sa[m] * sw[n] + bias[n])   (I8; F16 ignores sa/sw)
// A row-major (lda) or packed-A (a_packed, see common.hpp a_frag_off_*); only
// columns n < c_cols are stored to C (row stride c_ld); with kv != NULL the
// columns [hid, 3 hid) are appended to the KV pages instead (qkv projection).
struct WeightGemm {
  int dtype = LLM_I8;
  const void* A = nullptr;
  int lda = 0;
  int a_packed = 0;
  const void* W_packed = nullptr;
  int M = 0, N = 0, K = 0;
  const float* sa = nullptr;
  const float* sw = nullptr;
  const float* bias = nullptr;
  int act = LLM_ACT_NONE;
  float* C = nullptr;         // may be NULL when C16 is the only output
  int c_cols = 0, c_ld = 0;  // 0: N
  void* C16 = nullptr;       // fp16 copy of C in packed-A order with K = N (next GEMM's input)
  const KvAppendView* kv = nullptr;
  // LayerNorm prologue: A = LN(ln_x) (I8: quantised per row, the row scales
  // replace sa) computed per workgroup into LDS, when the rows' A image fits
  // (ln_fusable); act_out / sa_out optionally receive A (packed-A order) and
  // the row scales (activation taps).  A / sa are then ignored.
  const float* ln_x = nullptr;
  const _Float16* ln_emb = nullptr;  // optional: rows are E[ln_tok[m]] (fp16) instead of ln_x
  const int32_t* ln_tok = nullptr;
  int ln_V = 0;
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 1e-5f;
  void* act_out = nullptr;
  float* sa_out = nullptr;
  int w_keep = 0;  // weights with the default cache policy (kept in the Infinity Cache), else nt
  // I8: ln_x holds fp32 rows to quantise per row into A (no LayerNorm; ln_g /
  // ln_b unused) -- the o_proj prologue replacing the attention merge's
  // quantisation (quant_prologue_ok)
  int ln_quant_only = 0;
  // I8 only, act NONE: 1 = two k slices, each adding its dequantised half
  // (bias with slice 0) into C with one fp32 atomic add per element.  C must
  // hold zeros; with exactly two addends the sum is the same bits in either
  // order (0 + a = a, a + b = b + a), so the result is deterministic.
  int ksplit2 = 0;
};

// Input of a LayerNorm when it is not x: embedding rows E[tok[r]] (the decode
// step's first LayerNorm reads the token embedding directly, no embed launch).
struct LnSource {
  const _Float16* emb = nullptr;
  const int32_t* tok = nullptr;
  int V = 0;
  // optional (x rows only): the launch writes zeros over the rows it read,
  // once they are loaded (the next GEMM accumulates into them: ksplit2)
  float* zero_x = nullptr;
};

int weight_gemm(const WeightGemm& g, hipStream_t st);
// Whether weight_gemm can run the LayerNorm prologue for M rows of K (the
// per-workgroup A image must fit in LDS; K <= 128 groups of 16 bytes).
bool ln_fusable(int dtype, int M, int K);
// Whether weight_gemm can run the quantising prologue (ln_quant_only) for an
// I8 GEMM of M rows, N columns, K inputs.
bool quant_prologue_ok(int M, int N, int K);

}  // namespace llm
