// Decode-shaped weight GEMMs on gfx950 MFMA: the kernels and their launch
// forms (device code of gemm.hip, shared with the tuning build's
// csrc/tune/gemm_tune.hip).
//
//
//   i8_gemm : v_mfma_i32_16x16x64_i8, exact int32 accumulate, fp32 epilogue
//             (qkv_proj / o_proj / mlp_fc1 / mlp_fc2 of INT8Decoder; contract of
//             dnnl_matmul_int8, attention_cpu/dnnl_matmul_int8.cpp:7-75)
//   f16_gemm: v_mfma_f32_16x16x32_f16 (CUDADecoder weights; MLP<T>::forward,
//             decoder/mlp.hpp:23-41)
//
// Decode GEMMs have M = rows in flight (<= 64 per block) and stream every
// weight byte once: they are HBM-bound (128 op/B at M = 64 vs a ~625 op/B
// ridge).  So the design is a weight stream, not a compute tile:
//   * weights are repacked once at load time into MFMA B-fragment order:
//     for every (16-column tile, k-step) one contiguous 1 KiB block in which
//     lane l's 16 bytes are exactly its B operand -> one fully coalesced
//     buffer_load_dwordx4 per MFMA;
//   * a 512-thread workgroup owns one 16-column tile x up to 64 rows and its
//     8 waves split K; each wave issues 4 k-steps of loads before its MFMAs
//     (all of a decode GEMM's weight bytes are in flight at once), partial
//     accumulators are summed through LDS in a fixed order (deterministic),
//     then the fused dequant / bias / activation epilogue writes fp32.
//   * the k order inside a fragment (lane group l>>4 holds k = 16*(l>>4)+j) is
//     the same for A and B, so the dot product is exact whatever the
//     hardware's internal k permutation; C/D layout: col = lane&15,
//     row = 4*(lane>>4) + reg (cdna_hip_programming.md §3).
#pragma once

#include "common.hpp"
#include "gemm.hpp"
#include "ln_wave.hpp"

namespace llm {

// Optional epilogue target of the fused qkv projection: columns [hid, 2 hid)
// (K) and [2 hid, 3 hid) (V) of row m are written as fp16 into the page of
// position pos[m] (KVTileCache::get_write_ptr, kv_cache/kv_tile_cache.hpp:28-34)
// instead of a separate append launch.
struct KvAppend {
  const int32_t* pos;
  const int32_t* page_table;  // [num_beams][H][max_tiles] of this layer (row offset applied)
  const int32_t* rows;        // page-table row of GEMM row m (NULL: m) — prefill chunks
  _Float16* k_pool;
  _Float16* v_pool;
  int num_beams, max_tiles, TS, num_pages, H, D;
  size_t page_stride;  // elements from page p to page p + 1
};

struct GemmArgs {
  const uint8_t* A;
  int lda;            // elements
  int a_packed;       // 1: A is in MFMA A-fragment order (gemm_pack_weights of A^T), I8/F16
  const uint8_t* B;   // packed weights, or E rows for the LM head
  int M, N, K, KS;    // KS = number of k-steps
  const float* sa;
  const float* sw;
  const float* bias;
  int act;
  float* C;
  int32_t* acc_out;
  int c_cols;         // columns of C actually stored (< N with a KV append: q only)
  int c_ld;           // row stride of C
  _Float16* c16;      // optional fp16 copy of C in packed-A order (the next GEMM's input)
  KvAppend kv;        // kv.k_pool == nullptr: no append
  unsigned long long* stamps;  // diagnostics only (i8_gemm_stamps): per-workgroup phase clocks
  // LayerNorm prologue (gemm_kernel<..., PRO = 1>): A = LN(ln_x) (I8: quantised
  // per row, scales kept in LDS for the epilogue), computed by every workgroup
  // for its own rows into LDS instead of read from a LayerNorm launch's output
  const float* ln_x;      // [M][K] fp32
  const _Float16* ln_emb; // or rows E[ln_tok[m]] (fp16 [V][K])
  const int32_t* ln_tok;
  int ln_V;
  const float* ln_g;      // [K]
  const float* ln_b;      // [K]
  float ln_eps;
  uint8_t* act_out;       // optional: workgroups of column block 0 store A (packed-A order)
  float* sa_out;          //   and the I8 row scales (activation taps)
  // split-K (I8, gridDim.z = k slices; tuning build only, i8_gemm_tune_sk):
  // slice z sums k-steps [z KS/Z, (z+1) KS/Z) and stores its exact int32
  // partial sums to acc_out + z * M * N ([M][N]), nothing else.  The decode
  // step used it into the LayerNorm launch until round 3 (narrow_decode_tile).
  int partial;
  // 1: weights loaded with the default cache policy (a model whose weights fit
  // the 256 MiB Infinity Cache keeps them there from step to step); 0: nt
  // (streamed once per step, not kept: larger models)
  int w_keep;
  // split-K only (tuning build): 1 = workgroups remapped so that slice z runs on XCDs
  // [z 8/Z, (z+1) 8/Z) (dispatch places linear workgroup i on XCD i % 8), so
  // each XCD's L2 fetches only its slices' A columns instead of all of A
  // (launch_gemm checks 8 % Z == 0 and tiles * Z % 8 == 0)
  int xcd_map;
  // seam experiment (tuning build, gemm_pair_f16_kernel): arrival counter the
  // LayerNorm-prologue tile waits on after issuing its first weight batches
  unsigned* seam;
  int seam_n;
  int qdiag;  // tuning build, timing only: bit0 skip the prologue, bit1 no weight loads before it
  int ksplit2;  // WeightGemm::ksplit2: gridDim.z = 2, each slice atomically adds into C
};

// LDS image of A for the LayerNorm prologue: row-major 16-byte groups, row
// stride K * ESIZE + 32 bytes.  With that stride (K * ESIZE a multiple of 256)
// a wave writing one row is conflict-free (8 consecutive lanes = 128
// contiguous bytes) and the fragment read of a k-step (lane l: row l & 15,
// group 4 ks + (l >> 4)) puts every 16-lane ds_read_b128 group on 16
// distinct 16-byte slots (slot = 2 row + group mod 16).
__host__ __device__ constexpr int ln_row_stride(int K, int esize) { return K * esize + 32; }

// Phase clock (100 MHz s_memrealtime) of the diagnostic build path.
__device__ __forceinline__ unsigned long long phase_clock() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}


// k-steps per pipeline batch (two batches in flight): bounded by the VGPRs of
// the A fragments (MT tiles, x2 for the fp32 LM-head A) held per k-step.
template <int MT, int WAVES, int NT = 1>
constexpr int gemm_unroll() {
  // 4-wave workgroups carry twice the k-steps per wave: twice the batch, so
  // the same bytes are in flight from half the waves; 4 column tiles hold
  // twice the fragments per k-step, so half the k-steps
  return (MT >= 4 ? 2 : 4) * (WAVES == 4 ? 2 : 1) / (NT >= 4 ? 2 : 1);
}

__device__ __forceinline__ float apply_act(float y, int act) {
  if (act == LLM_ACT_RELU) return fmaxf(y, 0.f);
  if (act == LLM_ACT_GELU) return 0.5f * y * (1.f + erff(y * 0.70710678118654752f));
  return y;
}

enum class GemmKind { I8, F16 };

template <GemmKind KIND>
struct GemmTraits;
template <>
struct GemmTraits<GemmKind::I8> {
  static constexpr int KSTEP = 64, ESIZE = 1;
  using acc_t = i32x4;
  using elem_t = int32_t;
};
template <>
struct GemmTraits<GemmKind::F16> {
  static constexpr int KSTEP = 32, ESIZE = 2;
  using acc_t = f32x4;
  using elem_t = float;
};

// One workgroup = NT consecutive 16-column tiles x 16*MT rows; its 8 waves
// split the k-steps.  Per k-step a wave loads the A fragments of its MT row
// tiles ONCE and reuses them for all NT column tiles (A:B bytes = MT:NT from
// L2, instead of MT:1), and the k loop is software-pipelined in batches of
// kUnroll k-steps: batch i+1's loads are in flight while batch i's MFMAs run.
// Weight loads are non-temporal (each weight byte is read once per step).
// DIAG (diagnostics only, i8_gemm_stamps): bit 0 = no A loads (A reads as
// zero), bit 1 = no epilogue (wave 0 stores one word per workgroup).
// LayerNorm (+ int8 quantisation) of this workgroup's ROWS rows of ln_x into
// the LDS image of A (ln_row_stride) and, for I8, the row scales into sa_lds:
// ln_wave.hpp, bit-identical to the LayerNorm launch.  One wave per row (rows
// w, w + WAVES, ...), two rows' loads in flight; gamma / beta loaded once.
template <GemmKind KIND, int ROWS, int WAVES>
__device__ __forceinline__ void ln_prologue(const GemmArgs& a, int m0, uint8_t* alds,
                                            float* sa_lds) {
  constexpr int ESIZE = GemmTraits<KIND>::ESIZE;
  constexpr int CPL = 8;  // float4 chunks per lane (K <= 2048, ln_fusable)
  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int K = a.K;
  const int K4 = K >> 2;
  const int stride = ln_row_stride(K, ESIZE);
  // ln_g == NULL: quantise only (I8: the fp32 rows are the attention output,
  // the o_proj prologue replacing the merge launch's per-row quantisation)
  const bool do_ln = a.ln_g != nullptr;
  LnRow<CPL> gm, bt;
  ln_wave_load(a.ln_g, K4, do_ln, gm);
  ln_wave_load(a.ln_b, K4, do_ln, bt);
  for (int r0 = w; r0 < ROWS; r0 += 2 * WAVES) {
    LnRow<CPL> x[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = r0 + q * WAVES;
      const int m = m0 + r;
      const bool ok = r < ROWS && m < a.M;
      if (a.ln_emb)
        ln_wave_load_f16(ok ? ln_embed_row(a.ln_emb, a.ln_tok, m, a.ln_V, K) : a.ln_emb, K4, ok,
                         x[q]);
      else
        ln_wave_load(a.ln_x + (size_t)m * K, K4, ok, x[q]);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = r0 + q * WAVES;
      if (r >= ROWS) break;
      const bool mok = m0 + r < a.M;  // rows past M: zero A (their outputs are not stored)
      float am;
      if (do_ln) {
        am = ln_wave_compute(x[q], gm, bt, K, a.ln_eps);
      } else {
        am = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(x[q].v[j][e]));
        am = ln_wave_max(am);
      }
      uint8_t* rowp = alds + (size_t)r * stride;
      if constexpr (KIND == GemmKind::I8) {
        const float scale = 127.f / (am + 1e-6f);
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = 64 * j + lane;  // consecutive lanes, consecutive dwords
          if (c < K4)
            *reinterpret_cast<uint32_t*>(rowp + 4 * c) = mok ? ln_quant4(x[q].v[j], scale) : 0u;
        }
        if (lane == 0) sa_lds[r] = mok ? 1.0f / scale : 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = 64 * j + lane;
          if (c < K4)
            *reinterpret_cast<ln_f16x4*>(rowp + 8 * c) =
                mok ? ln_half4(x[q].v[j]) : ln_f16x4{0, 0, 0, 0};
        }
      }
    }
  }
}

// One workgroup's tile (column block bx, row block by, k slice bz of nz);
// gx = column blocks in the grid (diagnostic stamps only).
// Wait (one lane, relaxed polls with s_sleep, then an acquire fence; the
// workgroup barrier after it orders every wave's loads) until *ctr >= n.
// Bounded: a timeout sets ctr[2] and runs on; it never hangs.
__device__ __forceinline__ void seam_wait(unsigned* ctr, int n) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)n) {
      __builtin_amdgcn_s_sleep(8);
      if (++spins > (1u << 21)) {
        __hip_atomic_store(&ctr[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <GemmKind KIND, int MT, int NT, int WAVES, int DIAG = 0, int PRO = 0, int SEAM = 0>
__device__ __forceinline__ void gemm_tile(const GemmArgs& a, int bx, int by, int bz, int nz,
                                          int gx) {
  using Tr = GemmTraits<KIND>;
  using acc_t = typename Tr::acc_t;
  constexpr int KSTEP = Tr::KSTEP;
  constexpr int kUnroll = gemm_unroll<MT, WAVES, NT>();
  // Cross-wave partial sums, [wave][tile][reg][lane]: lane-fastest so both the
  // per-register stores and the epilogue's reads (consecutive threads =
  // consecutive columns = consecutive lanes) are bank-conflict free.  With the
  // LayerNorm prologue (PRO = 1) they live in dynamic LDS, over the A image
  // once the k loop is done.
  using elem_t = typename Tr::elem_t;
  using RedT = elem_t[MT * NT][4][64];
  extern __shared__ __attribute__((aligned(16))) uint8_t gemm_smem[];
  RedT* red;
  if constexpr (PRO == 0) {
    __shared__ elem_t red_static[WAVES][MT * NT][4][64];
    red = red_static;
  } else {
    red = reinterpret_cast<RedT*>(gemm_smem);
  }
  constexpr int ROWS_ = 16 * MT;
  const int a_stride = ln_row_stride(a.K, Tr::ESIZE);
  uint8_t* alds = gemm_smem;
  float* sa_lds = reinterpret_cast<float*>(gemm_smem + (size_t)ROWS_ * a_stride);

  const int lane = lane_id();
  const int w = wave_id_uniform();
  const int nt0 = bx * NT;
  const int m0 = by * 16 * MT;
  unsigned long long* stamp =
      a.stamps ? a.stamps + ((size_t)by * gx + bx) * 48 : nullptr;
  if (stamp && lane == 0) stamp[w] = phase_clock();  // [0, 16): wave start
  // Wave w streams k range wr = (w + bx) % WAVES: at any moment the
  // workgroups of an XCD read different A fragments (all of them read all of
  // A), instead of every workgroup hitting the same L2 lines.
  const int wr = (w + bx) % WAVES;
  const int kz0 = (int)((bz * a.KS) / nz);  // this k slice (split-K)
  const int kzn = (int)(((bz + 1) * a.KS) / nz) - kz0;
  const int ks0 = kz0 + (wr * kzn) / WAVES;
  const int ks1 = kz0 + ((wr + 1) * kzn) / WAVES;
  const int ntiles = (a.N + 15) >> 4;

  // A descriptor: rows >= M (and anything past the matrix) read as zero.
  // Row-major A: lane l reads row l&15, k = 16*(l>>4) + j of each k-step (16
  // rows x 64 B per instruction).  Packed A: each (16-row tile, k-step)
  // fragment is one contiguous 1 KiB block (one fully coalesced load).
  const int arow_lane = lane & 15;
  const int kgrp = lane >> 4;
  const bool apk = a.a_packed;
  const uint32_t a_bytes = apk ? (uint32_t)(((a.M + 15) / 16) * a.KS * 1024u)
                               : (uint32_t)((size_t)a.M * a.lda * Tr::ESIZE);
  const auto arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a_bytes, 0x00020000);
  const uint32_t a_kstride = apk ? 1024u : (uint32_t)(KSTEP * Tr::ESIZE);
  const uint32_t a_kgrp_off = apk ? 0u : (uint32_t)(kgrp * (KSTEP / 4) * Tr::ESIZE);
  uint32_t a_row_off[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = m0 + mt * 16 + arow_lane;
    a_row_off[mt] = row >= a.M ? 0xFFFFFFF0u
                    : apk ? (uint32_t)((((m0 >> 4) + mt) * a.KS) * 1024u + lane * 16)
                          : (uint32_t)((size_t)row * a.lda * Tr::ESIZE);
  }
  // B descriptor: this workgroup's NT packed column tiles
  const uint8_t* bbase = a.B + (size_t)nt0 * a.KS * 1024;
  const uint32_t b_bytes = (uint32_t)(min(NT, ntiles - nt0) * a.KS * 1024u);
  uint32_t b_lane_off[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) b_lane_off[j] = (uint32_t)j * a.KS * 1024u + lane * 16;
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, (short)0, b_bytes, 0x00020000);

  acc_t acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[mt][j] = acc_t{0, 0, 0, 0};

  struct Batch {
    u32x4 b[kUnroll][NT];
    u32x4 af[kUnroll][MT];
  };
  // do_a / do_b: the LayerNorm-prologue kernel issues a batch's weight loads
  // before the prologue and its (LDS) A fragments after it
  auto issue = [&](Batch& bt, int ks, bool do_a = true, bool do_b = true) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int kk = ks + u;
      const bool ok = kk < ks1;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if (!do_b) break;
        const uint32_t boff = ok ? b_lane_off[j] + (uint32_t)kk * 1024u : 0xFFFFFFF0u;
        bt.b[u][j] = a.w_keep ? __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff, 0, 0)
                              : __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff, 0, 2);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (!do_a) break;
        if constexpr (PRO != 0) {
          // fragment (row mt*16 + (l & 15), group 4 kk + (l >> 4)) of the LDS image
          const int r = mt * 16 + arow_lane;
          bt.af[u][mt] = ok ? *reinterpret_cast<const u32x4*>(alds + (size_t)r * a_stride +
                                                             16 * (4 * kk + kgrp))
                            : u32x4{0u, 0u, 0u, 0u};
          continue;
        }
        const uint32_t koff = (uint32_t)kk * a_kstride + a_kgrp_off;
        const uint32_t aoff = (ok && a_row_off[mt] != 0xFFFFFFF0u) ? a_row_off[mt] + koff : 0xFFFFFFF0u;
        if constexpr ((DIAG & 1) != 0)
          bt.af[u][mt] = u32x4{aoff, 0u, 0u, 0u};
        else
          bt.af[u][mt] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, aoff, 0, 0);
      }
    }
  };
  auto compute = [&](const Batch& bt) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if constexpr (KIND == GemmKind::I8) {
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[mt][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                __builtin_bit_cast(i32x4, bt.af[u][mt]), __builtin_bit_cast(i32x4, bt.b[u][j]),
                acc[mt][j], 0, 0, 0);
        } else if constexpr (KIND == GemmKind::F16) {
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                __builtin_bit_cast(f16x8, bt.af[u][mt]), __builtin_bit_cast(f16x8, bt.b[u][j]),
                acc[mt][j], 0, 0, 0);
        }
      }
    }
  };

  // Epilogue operands are independent of the accumulators: load them before
  // the k loop so their round trips (scales, bias, and for KV append the
  // dependent pos -> page-table chain) overlap the weight stream instead of
  // following it.  Thread t owns outputs t, t + NTHR, ... (col fastest).
  constexpr int ROWS = 16 * MT, COLS = 16 * NT, NTHR = WAVES * 64;
  constexpr int EPT = (ROWS * COLS + NTHR - 1) / NTHR;
  const KvAppend& kv = a.kv;
  const int hid = kv.H * kv.D;
  float e_scale[EPT], e_bias[EPT];
  int e_pos[EPT], e_br[EPT], e_page[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int o = threadIdx.x + e * NTHR;
    const int m = m0 + o / COLS;
    const int n = nt0 * 16 + o % COLS;
    const bool valid = o < ROWS * COLS && m < a.M && n < a.N;
    e_scale[e] = 1.f;
    if constexpr (KIND == GemmKind::I8) {
      if (!PRO && valid && a.sa) e_scale[e] *= a.sa[m];
      if (valid && a.sw) e_scale[e] *= a.sw[n];
    }
    e_bias[e] = valid && a.bias && (!a.ksplit2 || bz == 0) ? a.bias[n] : 0.f;
    const bool kvcol = valid && kv.k_pool && n >= hid;
    e_pos[e] = kvcol ? kv.pos[m] : -1;
    e_br[e] = kvcol ? (kv.rows ? kv.rows[m] : m) : -1;
  }

  Batch b0, b1;
  bool b1_pre = false;  // b1's weight loads already issued
  if constexpr (PRO != 0) {
    // the first two batches' weights are in flight while the prologue runs
    bool pre = true;
#if LLM_TUNING
    pre = (a.qdiag & 2) == 0;
#endif
    if (pre && ks0 < ks1) issue(b0, ks0, false, true);
    if (pre && ks0 + kUnroll < ks1) {
      issue(b1, ks0 + kUnroll, false, true);
      b1_pre = true;
    }
    if constexpr (SEAM != 0) seam_wait(a.seam, a.seam_n);  // weights already in flight
#if LLM_TUNING
    if ((a.qdiag & 1) == 0)
#endif
    ln_prologue<KIND, ROWS_, WAVES>(a, m0, alds, sa_lds);
    __syncthreads();
    if constexpr (KIND == GemmKind::I8) {
#pragma unroll
      for (int e = 0; e < EPT; ++e) {  // the prologue's row scales into the dequant factor
        const int o = threadIdx.x + e * NTHR;
        if (o < ROWS * COLS) e_scale[e] *= sa_lds[o / COLS];
      }
    }
    if (a.act_out && bx == 0) {  // activation taps: A in packed-A order + scales
      const int KS = a.KS;
      for (int i = threadIdx.x; i < ROWS_ * KS * 4; i += NTHR) {
        const int r = i / (KS * 4), g = i % (KS * 4);
        const int m = m0 + r;
        if (m >= a.M) continue;
        const size_t off = ((size_t)((m >> 4) * KS + (g >> 2)) * 64 + (m & 15) + 16 * (g & 3)) * 16;
        *reinterpret_cast<u32x4*>(a.act_out + off) =
            *reinterpret_cast<const u32x4*>(alds + (size_t)r * a_stride + 16 * g);
      }
      if (KIND == GemmKind::I8 && a.sa_out && threadIdx.x < ROWS_ && m0 + (int)threadIdx.x < a.M)
        a.sa_out[m0 + threadIdx.x] = sa_lds[threadIdx.x];
    }
  }

  {
    int ks = ks0;
    bool b0_b = PRO == 0;
#if LLM_TUNING
    if constexpr (PRO != 0) b0_b = (a.qdiag & 2) != 0;  // weights not issued before the prologue
#endif
    if (ks < ks1) issue(b0, ks, true, b0_b);
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int o = threadIdx.x + e * NTHR;
      const int n = nt0 * 16 + o % COLS;
      const int p = e_pos[e], br = e_br[e];
      int page = -1;
      if (p >= 0 && br >= 0 && br < kv.num_beams && p / kv.TS < kv.max_tiles) {
        const int which = n >= 2 * hid;
        const int h = (n - hid * (1 + which)) / kv.D;
        page = kv.page_table[((size_t)br * kv.H + h) * kv.max_tiles + p / kv.TS];
        if (page >= kv.num_pages) page = -1;
      }
      e_page[e] = page;
    }
    while (ks < ks1) {
      if (ks + kUnroll < ks1) {
        issue(b1, ks + kUnroll, true, !b1_pre);
        b1_pre = false;
      }
      compute(b0);
      ks += kUnroll;
      if (ks >= ks1) break;
      if (ks + kUnroll < ks1) issue(b0, ks + kUnroll);
      compute(b1);
      ks += kUnroll;
    }
  }

  if (stamp && lane == 0) stamp[16 + w] = phase_clock();  // [16, 32): k loop done
  if constexpr ((DIAG & 2) != 0) {
    int32_t x = 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NT; ++j) x ^= (int32_t)acc[mt][j][0] ^ (int32_t)acc[mt][j][3];
    if (lane == 0 && a.C) a.C[bx] = (float)x;
    if (stamp && lane == 0) stamp[32 + w] = phase_clock();
    return;
  }
  if constexpr (PRO != 0) __syncthreads();  // every wave is done with the A image
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wr][mt * NT + j][r][lane] = acc[mt][j][r];
  __syncthreads();

#pragma unroll
  for (int e = 0; e < EPT; ++e) {
#pragma clang fp contract(off)  // y = acc * scale + bias rounded twice, as the reference
    const int o = threadIdx.x + e * NTHR;
    if (o >= ROWS * COLS) break;
    const int cl = o % COLS;
    const int row = o / COLS;
    const int j = cl >> 4;
    const int col = cl & 15;
    const int mt = row >> 4;
    const int rl = row & 15;
    const int src_lane = (rl >> 2) * 16 + col;
    const int reg = rl & 3;
    const int m = m0 + row;
    const int n = (nt0 + j) * 16 + col;
    if (m >= a.M || n >= a.N) continue;
    float y;
    if constexpr (KIND == GemmKind::I8) {
      int32_t s = 0;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) s += red[ww][mt * NT + j][reg][src_lane];
#if LLM_TUNING
      if (a.partial) {
        a.acc_out[((size_t)bz * a.M + m) * a.N + n] = s;
        continue;
      }
#endif
      if (a.acc_out) a.acc_out[(size_t)m * a.N + n] = s;
      y = (float)s * e_scale[e];
      if (a.bias) y = y + e_bias[e];
      if (a.ksplit2) {  // this k slice's share (bias with slice 0), added into C
        atomicAdd(a.C + (size_t)m * a.c_ld + n, y);
        continue;
      }
    } else {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) s += red[ww][mt * NT + j][reg][src_lane];
      y = a.bias ? s + e_bias[e] : s;
    }
    y = apply_act(y, a.act);
    if (a.C && n < a.c_cols) a.C[(size_t)m * a.c_ld + n] = y;
    if (a.c16) a.c16[a_frag_off_f16(m, n, a.N >> 5)] = (_Float16)y;
    if (e_page[e] >= 0) {
      const int which = n >= 2 * hid;  // 0: K, 1: V
      const int i = n - hid * (1 + which);
      const int d = i % kv.D;
      const int p = e_pos[e];
      const size_t off = (size_t)e_page[e] * kv.page_stride + (size_t)(p % kv.TS) * kv.D + d;
      (which ? kv.v_pool : kv.k_pool)[off] = (_Float16)y;
    }
  }
  if (stamp && lane == 0) stamp[32 + w] = phase_clock();  // [32, 48): wave end
}

template <GemmKind KIND, int MT, int NT, int WAVES, int DIAG = 0, int PRO = 0>
__global__ __launch_bounds__(WAVES * 64) void gemm_kernel(GemmArgs a) {
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
#if LLM_TUNING
  if (a.xcd_map) {
    const int per = 8 / (int)gridDim.z;  // XCDs per k slice
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = lin & 7;
    const int tile = (lin >> 3) * per + xcd % per;
    bz = xcd / per;
    bx = tile % (int)gridDim.x;
    by = tile / (int)gridDim.x;
  }
#endif
  gemm_tile<KIND, MT, NT, WAVES, DIAG, PRO>(a, bx, by, bz, (int)gridDim.z, (int)gridDim.x);
}

// Repack W [K][N] (row-major) into per-(16-col tile, k-step) 1 KiB blocks,
// lane l's 16 bytes = W[k0 + (l>>4)*EPL + j][n0 + (l&15)], j < EPL
// (EPL = elements per lane: 16 int8 or 8 fp16); zero-padded past K / N.
template <typename T, int EPL>
__global__ void pack_kernel(const T* __restrict__ W, T* __restrict__ P, int K, int N, int KS,
                            int ntiles) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one lane-chunk
  const size_t total = (size_t)ntiles * KS * 64;
  if (idx >= total) return;
  const int lane = idx & 63;
  const size_t blk = idx >> 6;
  const int ks = blk % KS;
  const int nt = blk / KS;
  const int n = nt * 16 + (lane & 15);
  const int kb = ks * (4 * EPL) + (lane >> 4) * EPL;
  T* dst = P + idx * EPL;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int k = kb + j;
    dst[j] = (k < K && n < N) ? W[(size_t)k * N + n] : T(0);
  }
}

namespace {

// Column tiles per workgroup: 2 when that still leaves >= 192 workgroups
// (measured: qkv 9.9 vs 12.2 us, fc1 10.5 vs 12.5 us at M = 64), else 1.
// At <= 16 rows A is one 16-row fragment per k-step, so sharing it over two
// column tiles saves little and halves the workgroups streaming the weights:
// 1 (C3 shapes at M = 8, graph-replayed, profiles/r05/gemm_small_m.txt: qkv
// 5.28 -> 4.95 us, fc1 5.96 -> 5.25 us).
inline int pick_nt(int N, int M) {
  if (M <= 16) return 1;
  const int ntiles = (N + 15) / 16;
  const int mblocks = (M + 63) / 64;
  return (ntiles % 2 == 0 && (ntiles / 2) * mblocks >= 192) ? 2 : 1;
}

// Dynamic LDS of the LayerNorm-prologue kernel: the rows' A image + row
// scales, or the cross-wave partial sums that reuse it, whichever is larger.
template <GemmKind KIND, int MT, int NT, int WAVES>
size_t ln_lds_bytes(int K) {
  const size_t img = (size_t)16 * MT * ln_row_stride(K, GemmTraits<KIND>::ESIZE) + 16 * MT * 4;
  const size_t red = (size_t)WAVES * MT * NT * 4 * 64 * 4;
  return img > red ? img : red;
}
constexpr size_t kLnLdsMax = 160 * 1024;

template <GemmKind KIND, int MT, int NT>
hipError_t launch_gemm_nt(const GemmArgs& a, int waves, int mblocks, hipStream_t st, int kslices) {
  const int ntiles = (a.N + 15) / 16;
  const dim3 grid((ntiles + NT - 1) / NT, mblocks, kslices);
  if constexpr (NT <= 2) {
    if (a.ln_x) {
      const size_t lds = ln_lds_bytes<KIND, MT, NT, 8>(a.K);
      hipLaunchKernelGGL((gemm_kernel<KIND, MT, NT, 8, 0, 1>), grid, dim3(512), lds, st, a);
      return hipGetLastError();
    }
  }
  // the cross-wave sums' static LDS (WAVES x MT NT KiB) must stay <= 64 KiB
  if constexpr (MT * NT * 8 <= 64) {
    if (waves != 4) {
      hipLaunchKernelGGL((gemm_kernel<KIND, MT, NT, 8>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_kernel<KIND, MT, NT, 4>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

template <GemmKind KIND, int MT>
hipError_t launch_gemm_mt(const GemmArgs& a, int NT, int waves, int mblocks, hipStream_t st,
                          int kslices) {
#if LLM_TUNING
  if (NT == 4 && !a.ln_x) return launch_gemm_nt<KIND, MT, 4>(a, waves, mblocks, st, kslices);
  if (NT == 3 && !a.ln_x) return launch_gemm_nt<KIND, MT, 3>(a, waves, mblocks, st, kslices);
#endif
  return NT == 2 ? launch_gemm_nt<KIND, MT, 2>(a, waves, mblocks, st, kslices)
                 : launch_gemm_nt<KIND, MT, 1>(a, waves, mblocks, st, kslices);
}

}  // namespace

namespace {

// Waves per workgroup (they split K): 8.  The 4-wave form (twice the
// k-steps per wave) is kept for the tuning entry.
inline int pick_waves(const GemmArgs&, int) { return 8; }

// Decode rows 17..32 (C4's 32 beams): 16-row workgroups (each row block
// streams the weights; the repeat reads come from L2 / the Infinity Cache),
// 4-wave workgroups for K < 4096, in place of 32-row tiles and split-K.
// Graph-replayed sweep of every (NT, waves, rows) form (scripts/tune_gemm.py
// --M 32, two runs agree within 0.1 us): qkv 7.0 -> 6.5 us, o_proj 4.8 ->
// 3.6, fc2 10.1 -> 7.0 (fc1 keeps NT 2 x 32 rows, 7.8).  In the C4 step
// (same box, scripts/gpu_lib_ab.sh) +3.3..4.1 % over split-K.  At 64 rows
// (C3) the same forms lost 0.3 % to split-K.
// Decode rows 33..64 (C3), column grid under 256 tiles (o_proj, fc2 at hid
// 2048): 2 column tiles x 16 rows x 8 waves, four row blocks each streaming
// the weights (the repeats from L2 / the Infinity Cache).  Round 3 sweep of
// every (NT 1/2/4, waves, rows, k slices, XCD placement) form
// (scripts/tune_gemm_sk.py): o_proj 5.39 -> 4.74 us, fc2 9.74 -> 8.90 us
// against split-K 2 into the LayerNorm; in the C3 step (same box,
// scripts/gpu_lib_ab.sh, two rounds) 3,741 / 3,744 -> 3,811 / 3,802 tok/s,
// the LayerNorm launches also reading one fp32 row instead of two int32 slices.
// That retired split-K from the decode step (the tuning build keeps it).
struct TileChoice {
  int nt, waves, mrows;
};
// By shape: M rows, N columns, K inputs (the LayerNorm-prologue and split-K
// launches keep their own forms).
// Measured and not taken (round 3): C3's qkv (384 column tiles, 64 rows) as
// 3 column tiles x 32 rows x 8 waves (tuning build NT 3), 128 column blocks x
// 2 row blocks = 256 workgroups, each reading 96 KB of weights + 64 KB of A
// instead of 64 + 128 KB.  Standalone, weights from HBM (scripts/tune_gemm.py
// --nts 1 2 3, profiles/r03/gemm_nt3.txt) 9.32 -> 7.93 us, but in the C3 step
// (KV-append epilogue, same box, three rounds) 3,846-3,849 -> 3,840-3,845
// tok/s, parity green (profiles/r03/gemm_nt3_ab.txt).
inline bool narrow_tile_for(int M, int N, int K, TileChoice& t) {
  if (M <= 16 || M > 64) return false;
  const int ntiles = (N + 15) / 16;
  if (M > 32) {
    if (ntiles >= 256) return false;
    t = TileChoice{2, 8, 16};
    return true;
  }
  if (ntiles < 384) {
    t = K >= 4096 ? TileChoice{1, 8, 16} : TileChoice{1, 4, 16};
    return true;
  }
  if (ntiles < 512) {
    t = TileChoice{1, 4, 16};
    return true;
  }
  return false;
}
// fc2 as two k slices at 33..64 rows (decoder.cpp fc2_split: C5's K 16384):
// 2 column tiles x 64 rows x 8 waves per slice, 128 x 2 = 256 workgroups in
// one round, each reading half of A (512 KB instead of the 1-tile form's
// 1 MB per workgroup).  Same box, C5 (profiles/r06/c5_fc2_k2_ab.txt):
// 1,441.1 / 1,442.5 against 1,438.9 / 1,439.5 tok/s; one column tile per
// slice (512 workgroups, two rounds) 1,435.4 / 1,437.5.  At C3 (K 8192) no
// tile of it beats the one-slice 16-row form (profiles/r06/c3_fc2_k2_ab.txt),
// nor at C4's 32 rows (c4_fc2_k2_ab.txt).
inline bool narrow_decode_tile(const GemmArgs& a, int kstep, TileChoice& t) {
  if ((a.ln_x && a.ln_g) || a.partial) return false;
  if (a.ksplit2 && a.M > 32 && a.M <= 64) {
    t = TileChoice{2, 8, 64};
    return true;
  }
  return narrow_tile_for(a.M, a.N, a.KS * kstep, t);
}

template <GemmKind KIND>
hipError_t launch_gemm(const GemmArgs& a_in, hipStream_t st, int nt_override = 0,
                       int waves_override = 0, int mrows_override = 0, int ks_override = 0) {
  GemmArgs a = a_in;
  TileChoice tc{0, 0, 0};
  const bool narrow = nt_override == 0 && waves_override == 0 && mrows_override == 0 &&
                      narrow_decode_tile(a, GemmTraits<KIND>::KSTEP, tc);
  if (narrow) {
    nt_override = tc.nt;
    waves_override = tc.waves;
    mrows_override = tc.mrows;
  }
  const int NT = nt_override > 0 ? nt_override : pick_nt(a.N, a.M);
  const int waves = waves_override > 0 ? waves_override : pick_waves(a, NT);
  // rows per workgroup: 32 when the column grid alone cannot fill the CUs
  // (M = 64: o_proj 5.8 -> 4.5 us, mlp_fc2 13.0 -> 9.6 us; the second row
  // block re-reads the weights, mostly from the Infinity Cache)
  int mrows = a.M <= 16 ? 16 : a.M <= 32 ? 32 : 64;
  // no split-K: 32 rows per workgroup when the column grid alone cannot fill
  // the CUs (the second row block re-reads the weights, mostly from the
  // Infinity Cache); split-K fills them with k slices instead
  if (mrows == 64 && NT == 1 && (a.N + 15) / 16 < 256 && !a.ln_x && !a.partial) mrows = 32;
  if (mrows_override > 0) mrows = mrows_override;
  const int ks = a.partial ? std::max(1, ks_override) : a.ksplit2 ? 2 : 1;
  const int mblocks = (a.M + mrows - 1) / mrows;
  const int tiles = ((a.N + 15) / 16 + NT - 1) / NT * mblocks;
  if (a.xcd_map && (ks < 2 || 8 % ks != 0 || (tiles * ks) % 8 != 0)) a.xcd_map = 0;
  if (mrows == 16) return launch_gemm_mt<KIND, 1>(a, NT, waves, mblocks, st, ks);
  if (mrows == 32) return launch_gemm_mt<KIND, 2>(a, NT, waves, mblocks, st, ks);
  return launch_gemm_mt<KIND, 4>(a, NT, waves, mblocks, st, ks);
}

}  // namespace
}  // namespace llm
