// The FP16 decoder's fused MLP launch (csrc/mlp_fused.hip): LN2 -> fc1 (+b1,
// ReLU) -> fc2 (+b2) in one launch, slices of the inter dimension per
// workgroup, the fc2 partials summed in the counted int64 columns of
// common.hpp (oacc_term).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace llm {

struct MlpFusedArgs {
  const float* x;        // [M][hid] fp32, LN2's input
  const float* ln_g;     // [hid]
  const float* ln_b;     // [hid]
  float eps;
  const uint8_t* w1;     // fc1 weights, packed fp16 B fragments [inter/16][hid/32][1 KiB]
  const float* b1;       // [inter]
  const uint8_t* w2;     // fc2 weights, packed [hid/16][inter/32][1 KiB]
  const float* b2;       // [hid]
  long long* acc;        // [M][hid] counted columns, zero between launches (left zero)
  float* out;            // [M][hid] y (x of the next layer; may alias x only if no
                         // other reader: the launch reads x in its prologue first)
  int* flag;             // set to 1 when a slice's term was clamped (oacc_term)
  uint8_t* act_out;      // optional tap: LN2 rows, packed-A fp16 [16][hid]
  _Float16* h_out;       // optional tap: fc1 output, packed-A fp16 [16][inter]
  int M, hid, inter;
  int nslice;            // inter / (16 * slice_tiles) workgroups
  int w_keep;            // weights with the default cache policy (else nt)
};

// Rows, widths and slice width (fc1 column tiles per workgroup: 2, 4 or 8)
// the fused launch takes: M <= 16, hid a multiple of 128 up to 1024 (768 at
// 8 tiles), 2..127
// slices.
bool mlp_fusable(int M, int hid, int inter, int slice_tiles);
hipError_t launch_mlp_f16_fused(const MlpFusedArgs& a, int slice_tiles, hipStream_t st);

}  // namespace llm
