// Tuning build only (make tune -> libllm_decoder_hip_tune.so; never in
// libllm_decoder_hip.so): GEMM entries with forced tile forms, split-K
// slices, phase clocks and the one-launch seam experiment, for the scripts
// that price them (scripts/tune_gemm*.py, gemm_phases.py, seam_pair.py) and
// the tile-form exactness tests (tests/test_gemm_gpu.py).
#include "gemm_impl.hpp"

using namespace llm;

// Tuning hook (not in include/llm_decoder.h): i8_gemm with a forced column-tile
// count, waves per workgroup and rows per workgroup (16 / 32 / 64; 0 = auto).
// Diagnostic (not in include/llm_decoder.h): i8_gemm_tune with per-workgroup
// phase clocks, stamps[wg][0..16) wave start, [16..32) k loop done, [32..48) wave end, plus one
// launch-end clock per workgroup in ends[wg] (100 MHz ticks).
__global__ void gemm_end_stamp_kernel(unsigned long long* t) {
  if (threadIdx.x == 0) *t = phase_clock();
}

extern "C" int i8_gemm_stamps(int nt, int waves, int mrows, const int8_t* A, const void* W_packed,
                              float* C, int M, int N, int K, const float* sa, const float* sw,
                              unsigned long long* stamps, unsigned long long* end_stamp,
                              void* stream) {
  GemmArgs a{};
  a.a_packed = 1;
  a.A = reinterpret_cast<const uint8_t*>(A);
  a.lda = K;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.sa = sa; a.sw = sw; a.C = C; a.c_cols = N; a.c_ld = N;
  a.stamps = stamps;
  hipStream_t st = as_stream(stream);
  hipError_t e = hipSuccess;
  const int ntiles = N / 16;
  const int diag = waves >> 8;  // waves = 8 | (diag << 8)
  if (diag == 0) {
    e = launch_gemm<GemmKind::I8>(a, st, nt, waves, mrows);
  } else {
    // diagnostic forms of the two production shapes only
    LLM_REQUIRE((nt == 2 && mrows == 64) || (nt == 1 && mrows == 32), "i8_gemm_stamps: diag shape");
    auto go = [&](auto kern, int NTv, int mr) {
      hipLaunchKernelGGL(kern, dim3((ntiles + NTv - 1) / NTv, (M + mr - 1) / mr), dim3(512), 0, st, a);
    };
    if (nt == 2) {
      if (diag == 1) go(gemm_kernel<GemmKind::I8, 4, 2, 8, 1>, 2, 64);
      else if (diag == 2) go(gemm_kernel<GemmKind::I8, 4, 2, 8, 2>, 2, 64);
      else go(gemm_kernel<GemmKind::I8, 4, 2, 8, 3>, 2, 64);
    } else {
      if (diag == 1) go(gemm_kernel<GemmKind::I8, 2, 1, 8, 1>, 1, 32);
      else if (diag == 2) go(gemm_kernel<GemmKind::I8, 2, 1, 8, 2>, 1, 32);
      else go(gemm_kernel<GemmKind::I8, 2, 1, 8, 3>, 1, 32);
    }
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(gemm_end_stamp_kernel, dim3(1), dim3(64), 0, st, end_stamp);
    e = hipGetLastError();
  }
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "i8_gemm_stamps");
}

extern "C" int i8_gemm_tune(int nt, int waves, int mrows, int a_packed, const int8_t* A, int lda,
                            const void* W_packed, float* C, int M, int N, int K, const float* sa,
                            const float* sw, void* stream) {
  GemmArgs a{};
  a.a_packed = a_packed;
  a.A = reinterpret_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.sa = sa; a.sw = sw; a.C = C; a.c_cols = N; a.c_ld = N;
  hipError_t e = launch_gemm<GemmKind::I8>(a, as_stream(stream), nt, waves, mrows);
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "i8_gemm_tune");
}

// The quantising prologue as the decoder's o_proj runs it (weight_gemm with
// ln_quant_only): fp32 rows x [M][K] quantised per row in the prologue, the
// product-path tile choice; for timing against i8_gemm_tune on packed int8 A.
extern "C" int i8_gemm_tune_qpro(const float* x, const void* W_packed, float* C, int M, int N,
                                 int K, const float* sw, int qdiag, void* stream) {
  LLM_REQUIRE(quant_prologue_ok(M, N, K), "i8_gemm_tune_qpro: shape");
  GemmArgs a{};
  a.a_packed = 1;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.sw = sw; a.C = C; a.c_cols = N; a.c_ld = N;
  a.ln_x = x;  // ln_g NULL: the quantising prologue
  a.ln_eps = 1e-5f;
  a.qdiag = qdiag;
  hipError_t e = launch_gemm<GemmKind::I8>(a, as_stream(stream));
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "i8_gemm_tune_qpro");
}

// Split-K forms: int32 partial slices only (acc_out [kslices][M][N]), packed A;
// xcd_map as GemmArgs::xcd_map (ignored where the grid does not allow it).
extern "C" int i8_gemm_tune_sk(int nt, int waves, int mrows, int kslices, int xcd_map,
                               const int8_t* A, const void* W_packed, int32_t* acc_out, int M,
                               int N, int K, void* stream) {
  LLM_REQUIRE(kslices >= 1 && kslices <= 8 && K % 64 == 0 && N % 16 == 0, "i8_gemm_tune_sk: shape");
  GemmArgs a{};
  a.a_packed = 1;
  a.A = reinterpret_cast<const uint8_t*>(A);
  a.lda = K;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.partial = 1;
  a.acc_out = acc_out;
  a.xcd_map = xcd_map;
  hipError_t e = launch_gemm<GemmKind::I8>(a, as_stream(stream), nt, waves, mrows, kslices);
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "i8_gemm_tune_sk");
}

// Seam experiment (round 3, the C2 verdict item): o_proj -> LN2 + fc1 of the
// FP16 decoder at <= 16 rows as ONE launch, workgroups 0..n1-1 computing the
// o_proj tiles, then every workgroup waiting on a device-scope arrival counter
// (release fence + agent-scope add; relaxed poll with s_sleep, bounded: a
// timeout sets sync[2] and runs on, it never hangs) before its fc1 tile with
// the LayerNorm prologue.  sync[0..2] self-reset (the last departing
// workgroup clears them).  Against the decoder's two launches of the same
// tile forms: f16_gemm_pair_tune(fused = 0 / 1).
__global__ __launch_bounds__(512) void gemm_pair_f16_kernel(GemmArgs a1, GemmArgs a2, int n1,
                                                            unsigned* sync) {
  const int wg = blockIdx.x;
  if (wg < n1) {
    gemm_tile<GemmKind::F16, 1, 1, 8, 0, 0>(a1, wg, 0, 0, 1, n1);
    // every wave's stores done (the barrier waits on them), then ONE release
    // fence for the workgroup (one per wave: 19.2 us per pair) and the add
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // fc1 tile: its first weight batches issued, then seam_wait, then the
  // LayerNorm prologue reads the o_proj rows
  gemm_tile<GemmKind::F16, 1, 1, 8, 0, 1, 1>(a2, wg, 0, 0, 1, (int)gridDim.x);
  // departure: the last workgroup out clears the counters for the next launch
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(&sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

extern "C" int f16_gemm_pair_tune(const void* A1, const void* W1, float* x, const float* ln_g,
                                  const float* ln_b, const void* W2, const float* b2, void* C16,
                                  int M, int K, int N1, int N2, unsigned* sync, int fused,
                                  void* stream) {
  LLM_REQUIRE(M >= 1 && M <= 16 && K == N1 && K % 32 == 0 && N1 % 16 == 0 && N2 % 32 == 0 &&
                  ln_fusable(LLM_F16, M, K) && N2 / 16 >= N1 / 16 && N2 / 16 <= 256,
              "f16_gemm_pair_tune: shape");
  GemmArgs a1{};
  a1.a_packed = 1;
  a1.A = static_cast<const uint8_t*>(A1);
  a1.B = static_cast<const uint8_t*>(W1);
  a1.M = M; a1.N = N1; a1.K = K; a1.KS = K / 32;
  a1.C = x; a1.c_cols = N1; a1.c_ld = N1;
  a1.w_keep = 1;  // as the C2 decoder (its weights fit the Infinity Cache)
  GemmArgs a2{};
  a2.a_packed = 1;
  a2.B = static_cast<const uint8_t*>(W2);
  a2.M = M; a2.N = N2; a2.K = N1; a2.KS = N1 / 32;
  a2.bias = b2; a2.act = LLM_ACT_RELU;
  a2.c16 = static_cast<_Float16*>(C16);
  a2.c_cols = 0; a2.c_ld = N2;
  a2.ln_x = x; a2.ln_g = ln_g; a2.ln_b = ln_b; a2.ln_eps = 1e-5f;
  a2.w_keep = 1;
  a2.seam = sync;
  a2.seam_n = N1 / 16;
  hipStream_t st = as_stream(stream);
  hipError_t e;
  if (!fused) {
    e = launch_gemm<GemmKind::F16>(a1, st);
    if (e == hipSuccess) e = launch_gemm<GemmKind::F16>(a2, st);
  } else {
    const size_t lds = ln_lds_bytes<GemmKind::F16, 1, 1, 8>(N1);
    hipLaunchKernelGGL(gemm_pair_f16_kernel, dim3(N2 / 16), dim3(512), lds, st, a1, a2, N1 / 16,
                       sync);
    e = hipGetLastError();
  }
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "f16_gemm_pair_tune");
}

// The FP16 GEMM with a forced form (A in packed-A order when a_packed).
extern "C" int f16_gemm_tune(int nt, int waves, int mrows, int a_packed, const void* A, int lda,
                             const void* W_packed, float* C, int M, int N, int K, void* stream) {
  GemmArgs a{};
  a.a_packed = a_packed;
  a.A = static_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 32;
  a.C = C; a.c_cols = N; a.c_ld = N;
  hipError_t e = launch_gemm<GemmKind::F16>(a, as_stream(stream), nt, waves, mrows);
  return e == hipSuccess ? LLM_OK : fail(LLM_ERR_HIP, "f16_gemm_tune");
}
