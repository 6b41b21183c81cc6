// The FP16 decoder's MLP in ONE launch, no grid barrier (MLP<T>::forward,
// decoder/mlp.hpp:23-41, after LN2: y = ReLU(LN2(x) W1 + b1) W2 + b2).
//
// Decode rows are few (<= 16) and the two weight matrices are the whole cost
// (C2: 4.7 MB each), so the launch is a weight stream cut by slices of the
// inter dimension: workgroup j owns inter columns J = [16 SJ j, 16 SJ (j+1)).
//   1. LN2 of the rows into an LDS A image (gemm_impl.hpp ln_prologue, the
//      fc1 GEMM's own prologue);
//   2. h_J = ReLU(A W1[:, J] + b1[J]): the 8 waves split the k-steps (the
//      fc1 GEMM's partition and fixed-order cross-wave sum, so h_J is the bits
//      fc1's epilogue writes), rounded to fp16 into a second LDS image (the
//      fc2 GEMM's packed fp16 input, the same rounding);
//   3. y_J = h_J W2[J, :]: every wave takes hid/128 of the output column
//      tiles over the slice's SJ/2 k-steps, and adds y_J into the counted
//      int64 columns of common.hpp (oacc_term: 2^56 per arrival + the value
//      in units of 2^-32).  Integer adds are order independent, so the sum is
//      the same bits whatever order the slices land in; the add whose returned
//      old value counts nslice - 1 arrivals completes the column: it stores
//      out[m][n] = sum + b2[n] and clears the column for the next launch.
// Every weight byte is read once; both weight streams are issued before the
// LayerNorm so their round trips overlap it.  The atomics are the price of the
// missing barrier: 16 x hid int64 per workgroup (MI355X_MICROARCH.md, global
// atomics ~1.3 TB/s of added bytes), so slices are wide (few workgroups).
#include "gemm_impl.hpp"
#include "mlp_fused.hpp"

namespace llm {

namespace {

constexpr int kMlpWaves = 8;

// LDS: the LN2 A image (16 rows, ln_row_stride) | cross-wave sums
// [8][SJ][4][64] fp32 | the h_J image [16][16 SJ + 8] fp16
template <int SJ>
constexpr size_t mlp_lds_bytes(int hid) {
  return (size_t)16 * ln_row_stride(hid, 2) + (size_t)kMlpWaves * SJ * 1024 +
         (size_t)16 * (16 * SJ + 8) * 2;
}

// SJ: fc1 column tiles per workgroup (slice width 16 SJ); KW1: fc1 k-steps per
// wave (hid / 256 rounded up); TPW: fc2 column tiles per wave (hid / 128)
template <int SJ, int KW1, int TPW>
__global__ __launch_bounds__(512) void mlp_f16_fused_kernel(MlpFusedArgs a) {
  static_assert(SJ % 2 == 0, "a slice is whole fc2 k-steps (32 inter columns)");
  constexpr int KL = SJ / 2;  // fc2 k-steps of the slice
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int j = blockIdx.x;
  const int hid = a.hid;
  const int KS1 = hid >> 5;           // fc1 k-steps
  const int KS2 = a.inter >> 5;       // fc2 k-steps (all of inter)
  const int NT2 = hid >> 4;           // fc2 column tiles
  const int a_stride = ln_row_stride(hid, 2);
  uint8_t* alds = smem;
  float* red = reinterpret_cast<float*>(smem + (size_t)16 * a_stride);  // [8][SJ][4][64]
  _Float16* hlds = reinterpret_cast<_Float16*>(smem + (size_t)16 * a_stride + kMlpWaves * SJ * 1024);
  constexpr int HST = 16 * SJ + 8;    // h image row stride (halves)

  // fc1: this workgroup's SJ column tiles; wave w sums k range wr (the fc1
  // GEMM's rotation, so the ranges are summed in the same order)
  const int wr = (w + j) % kMlpWaves;
  const int ks0 = (wr * KS1) / kMlpWaves, ks1 = ((wr + 1) * KS1) / kMlpWaves;
  const int aux = a.w_keep ? 0 : 2;
  const uint8_t* w1 = a.w1 + (size_t)j * SJ * KS1 * 1024;
  const auto r1 = __builtin_amdgcn_make_buffer_rsrc((void*)w1, (short)0,
                                                    (uint32_t)(SJ * KS1 * 1024), 0x00020000);
  // fc2: wave w takes column tiles w, w + 8, ... of hid/16; the slice's k-steps
  const int ntw = (NT2 - w + kMlpWaves - 1) / kMlpWaves;
  const uint8_t* w2 = a.w2 + (size_t)j * KL * 1024;
  const auto r2 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)w2, (short)0, (uint32_t)(((size_t)(NT2 - 1) * KS2 + KL) * 1024), 0x00020000);

  // the fc1 weights in flight before the LayerNorm (zero-record loads past the
  // wave's share: no bytes); the fc2 weights follow once fc1's registers are free
  u32x4 b1v[KW1][SJ];
#pragma unroll
  for (int u = 0; u < KW1; ++u)
#pragma unroll
    for (int t = 0; t < SJ; ++t) {
      const int ks = ks0 + u;
      const uint32_t off = ks < ks1 ? (uint32_t)((t * KS1 + ks) * 1024 + lane * 16) : 0xFFFFFFF0u;
      b1v[u][t] = aux ? __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, 2)
                      : __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, 0);
    }
  const int M = a.M;

  // 1. LN2 into the A image (rows >= M zero)
  {
    GemmArgs g{};
    g.M = M;
    g.K = hid;
    g.ln_x = a.x;
    g.ln_g = a.ln_g;
    g.ln_b = a.ln_b;
    g.ln_eps = a.eps;
    ln_prologue<GemmKind::F16, 16, kMlpWaves>(g, 0, alds, nullptr);
  }
  __syncthreads();
  if (a.act_out && j == 0) {  // activation tap: LN2 rows in packed-A order
    for (int i = threadIdx.x; i < 16 * KS1 * 4; i += 512) {
      const int r = i / (KS1 * 4), gg = i % (KS1 * 4);
      if (r >= M) continue;
      const size_t off = ((size_t)(gg >> 2) * 64 + r + 16 * (gg & 3)) * 16;
      *reinterpret_cast<u32x4*>(a.act_out + off) =
          *reinterpret_cast<const u32x4*>(alds + (size_t)r * a_stride + 16 * gg);
    }
  }

  // 2. fc1 slice
  f32x4 acc1[SJ];
#pragma unroll
  for (int t = 0; t < SJ; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = lane & 15, kgrp = lane >> 4;
#pragma unroll
  for (int u = 0; u < KW1; ++u) {
    const int ks = ks0 + u;
    if (ks >= ks1) break;
    const f16x8 af = __builtin_bit_cast(
        f16x8, *reinterpret_cast<const u32x4*>(alds + (size_t)arow * a_stride + 16 * (4 * ks + kgrp)));
#pragma unroll
    for (int t = 0; t < SJ; ++t)
      acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, __builtin_bit_cast(f16x8, b1v[u][t]),
                                                       acc1[t], 0, 0, 0);
  }
  u32x4 b2v[TPW][KL];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int nt = w + kMlpWaves * i;
      const uint32_t off =
          i < ntw ? (uint32_t)(((size_t)nt * KS2 + k) * 1024 + lane * 16) : 0xFFFFFFF0u;
      b2v[i][k] = aux ? __builtin_amdgcn_raw_buffer_load_b128(r2, off, 0, 2)
                      : __builtin_amdgcn_raw_buffer_load_b128(r2, off, 0, 0);
    }
#pragma unroll
  for (int t = 0; t < SJ; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((wr * SJ + t) * 4 + r) * 64 + lane] = acc1[t][r];
  __syncthreads();
  // h_J = ReLU(sum + b1) as fp16: thread o -> (row o / (16 SJ), column o % (16 SJ))
  for (int o = threadIdx.x; o < 16 * 16 * SJ; o += 512) {
    const int row = o / (16 * SJ), cl = o % (16 * SJ);
    const int t = cl >> 4, col = cl & 15;
    const int src = (row >> 2) * 16 + col, reg = row & 3;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < kMlpWaves; ++ww) s += red[((ww * SJ + t) * 4 + reg) * 64 + src];
    const int n1 = j * 16 * SJ + cl;
    const float y = fmaxf(s + a.b1[n1], 0.f);
    const _Float16 h = row < M ? (_Float16)y : (_Float16)0.f;
    hlds[row * HST + cl] = h;
    if (a.h_out && row < M) a.h_out[a_frag_off_f16(row, n1, KS2)] = h;  // fc1 tap
  }
  __syncthreads();

  // 3. fc2 partial of the slice into the counted columns
  f16x8 hf[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k)
    hf[k] = *reinterpret_cast<const f16x8*>(hlds + arow * HST + 32 * k + 8 * kgrp);
  const float lim = oacc_limit(a.nslice);
  bool clamped = false;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (i >= ntw) break;
    const int nt = w + kMlpWaves * i;
    f32x4 acc2 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KL; ++k)
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[k], __builtin_bit_cast(f16x8, b2v[i][k]),
                                                    acc2, 0, 0, 0);
    // lane: column 16 nt + (lane & 15), rows 4 (lane >> 4) + r
    const int n = nt * 16 + (lane & 15);
    long long tj[4], oj[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * kgrp + r;
      bool c;
      tj[r] = oacc_term(acc2[r], lim, c);
      clamped |= c && m < M;
      oj[r] = m < M ? (long long)atomicAdd(
                          reinterpret_cast<unsigned long long*>(a.acc + (size_t)m * hid + n),
                          (unsigned long long)tj[r])
                    : 0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * kgrp + r;
      if (m < M && oacc_count(oj[r]) == a.nslice - 1) {
        a.out[(size_t)m * hid + n] = oacc_value(oj[r] + tj[r]) + a.b2[n];
        __hip_atomic_store(a.acc + (size_t)m * hid + n, 0LL, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (clamped) *a.flag = 1;
}


// Slice widths (fc1 column tiles per workgroup) and the register shapes of
// the two row widths built: hid <= 768 (C2) and hid <= 1024.
template <int SJ>
hipError_t launch_sj(const MlpFusedArgs& a, hipStream_t st) {
  const size_t lds = mlp_lds_bytes<SJ>(a.hid);
  if (a.hid <= 768) {
    hipLaunchKernelGGL((mlp_f16_fused_kernel<SJ, 3, 6>), dim3(a.nslice), dim3(512), lds, st, a);
  } else {
    if constexpr (SJ <= 4)  // (8 tiles at hid 1024 would spill: mlp_fusable refuses it)
      hipLaunchKernelGGL((mlp_f16_fused_kernel<SJ, 4, 8>), dim3(a.nslice), dim3(512), lds, st, a);
  }
  return hipGetLastError();
}

}  // namespace

bool mlp_fusable(int M, int hid, int inter, int slice_tiles) {
  if (slice_tiles != 2 && slice_tiles != 4 && slice_tiles != 8) return false;
  const int w = 16 * slice_tiles;
  return M >= 1 && M <= 16 && hid % 128 == 0 && hid <= (slice_tiles == 8 ? 768 : 1024) &&
         inter % w == 0 && inter / w >= 2 && inter / w <= 127;
}

hipError_t launch_mlp_f16_fused(const MlpFusedArgs& a, int slice_tiles, hipStream_t st) {
  if (!mlp_fusable(a.M, a.hid, a.inter, slice_tiles) || a.nslice != a.inter / (16 * slice_tiles))
    return hipErrorInvalidValue;
  switch (slice_tiles) {
    case 2: return launch_sj<2>(a, st);
    case 4: return launch_sj<4>(a, st);
    default: return launch_sj<8>(a, st);
  }
}

}  // namespace llm
