// Decode-shaped weight GEMMs on gfx950 MFMA: the C entry points (i8_gemm,
// f16_gemm, gemm_pack_weights) and the decoder's weight_gemm.  Kernels, tile
// forms and design notes: gemm_impl.hpp; the tuning build's forced-form and
// diagnostic entries: csrc/tune/gemm_tune.hip.
#include "gemm_impl.hpp"

using namespace llm;

extern "C" size_t gemm_packed_bytes(int dtype, int K, int N) {
  if (K <= 0 || N <= 0) return 0;
  const int kstep = dtype == LLM_I8 ? 64 : 32;
  const size_t KS = (size_t)(K + kstep - 1) / kstep;
  const size_t nt = (size_t)(N + 15) / 16;
  return nt * KS * 1024;
}

extern "C" int gemm_pack_weights(int dtype, const void* W_kn, void* W_packed, int K, int N,
                                 void* stream) {
  LLM_REQUIRE(W_kn && W_packed && K > 0 && N > 0, "gemm_pack_weights: bad arguments");
  LLM_REQUIRE(dtype == LLM_I8 || dtype == LLM_F16, "gemm_pack_weights: dtype must be I8 or F16");
  const int kstep = dtype == LLM_I8 ? 64 : 32;
  const int KS = (K + kstep - 1) / kstep;
  const int ntiles = (N + 15) / 16;
  const size_t total = (size_t)ntiles * KS * 64;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = as_stream(stream);
  if (dtype == LLM_I8)
    hipLaunchKernelGGL((pack_kernel<int8_t, 16>), grid, dim3(256), 0, st,
                       static_cast<const int8_t*>(W_kn), static_cast<int8_t*>(W_packed), K, N, KS,
                       ntiles);
  else
    hipLaunchKernelGGL((pack_kernel<uint16_t, 8>), grid, dim3(256), 0, st,
                       static_cast<const uint16_t*>(W_kn), static_cast<uint16_t*>(W_packed), K, N,
                       KS, ntiles);
  LLM_HIP_RET(hipGetLastError());
  return LLM_OK;
}

extern "C" int i8_gemm(const int8_t* A, int lda, const void* W_packed, int32_t* acc_out, float* C,
                       int M, int N, int K, const float* sa, const float* sw, const float* bias,
                       int act, void* stream) {
  LLM_REQUIRE(M >= 0 && N > 0 && K > 0, "i8_gemm: bad M/N/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(A && W_packed, "i8_gemm: NULL operand");
  LLM_REQUIRE(K % 64 == 0, "i8_gemm: K must be a multiple of 64");
  LLM_REQUIRE(N % 16 == 0, "i8_gemm: N must be a multiple of 16");
  LLM_REQUIRE(lda >= K && lda % 16 == 0, "i8_gemm: lda must be >= K and a multiple of 16");
  LLM_REQUIRE(act >= 0 && act <= 2, "i8_gemm: bad activation");
  LLM_REQUIRE((size_t)M * lda < (1ull << 31), "i8_gemm: A too large");
  GemmArgs a{};
  a.A = reinterpret_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 64;
  a.sa = sa; a.sw = sw; a.bias = bias; a.act = act;
  a.C = C; a.acc_out = acc_out; a.c_cols = N; a.c_ld = N;
  hipError_t e = launch_gemm<GemmKind::I8>(a, as_stream(stream));
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("i8_gemm: ") + hipGetErrorString(e));
  return LLM_OK;
}

extern "C" int f16_gemm(const void* A, int lda, const void* W_packed, float* C, int M, int N,
                        int K, const float* bias, int act, void* stream) {
  LLM_REQUIRE(M >= 0 && N > 0 && K > 0, "f16_gemm: bad M/N/K");
  if (M == 0) return LLM_OK;
  LLM_REQUIRE(A && W_packed && C, "f16_gemm: NULL operand");
  LLM_REQUIRE(K % 32 == 0, "f16_gemm: K must be a multiple of 32");
  LLM_REQUIRE(N % 16 == 0, "f16_gemm: N must be a multiple of 16");
  LLM_REQUIRE(lda >= K && lda % 8 == 0, "f16_gemm: lda must be >= K and a multiple of 8");
  LLM_REQUIRE(act >= 0 && act <= 2, "f16_gemm: bad activation");
  LLM_REQUIRE((size_t)M * lda * 2 < (1ull << 31), "f16_gemm: A too large");
  GemmArgs a{};
  a.A = static_cast<const uint8_t*>(A);
  a.lda = lda;
  a.B = static_cast<const uint8_t*>(W_packed);
  a.M = M; a.N = N; a.K = K; a.KS = K / 32;
  a.bias = bias; a.act = act; a.C = C; a.c_cols = N; a.c_ld = N;
  hipError_t e = launch_gemm<GemmKind::F16>(a, as_stream(stream));
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("f16_gemm: ") + hipGetErrorString(e));
  return LLM_OK;
}


// The prologue pays off only while the fp32 rows every workgroup reads stay
// small: all workgroups read all of them, and a CU takes in L2-resident data
// at only ~80-120 GB/s (scripts/micro/bcast_read.hip: 256 KB per workgroup
// +2.2 us, 512 KB +6.4 us).  Same-box A/B of the decode step
// (scripts/gpu_ab.sh): C2 (16 rows x 768, 48 KB) +1.5-5 %; C4 (32 x 2048,
// 256 KB) -7 %; C3 (64 x 2048, 512 KB) -4 %.  So: at most 64 KB of rows.
bool llm::ln_fusable(int dtype, int M, int K) {
  const int es = dtype == LLM_I8 ? 1 : 2;
  if (K % 16 != 0 || (K * es) % 256 != 0 || K > 2048) return false;
  const int rows = M <= 16 ? 16 : M <= 32 ? 32 : 64;
  if ((size_t)rows * K * sizeof(float) > 64 * 1024) return false;
  return (size_t)rows * (ln_row_stride(K, es) + 4) <= kLnLdsMax;
}

// The quantising prologue (I8 o_proj reading the attention's fp32 rows): the
// workgroup's rows as the launch will tile them -- 16 at <= 16 rows and in
// the 16-row forms of 17..64 rows (narrow_decode_tile) -- at most 128 KB of
// fp32 read per workgroup and an int8 image that fits LDS.
bool llm::quant_prologue_ok(int M, int N, int K) {
  if (M <= 0 || M > 64 || K % 256 != 0 || K > 2048 || N % 16 != 0) return false;
  TileChoice t{0, 0, 0};
  const int rows = M <= 16 ? 16 : narrow_tile_for(M, N, K, t) ? t.mrows : 0;
  if (rows != 16) return false;
  return (size_t)rows * K * sizeof(float) <= 128 * 1024 &&
         (size_t)rows * (ln_row_stride(K, 1) + 4) <= kLnLdsMax;
}

int llm::weight_gemm(const WeightGemm& g, hipStream_t st) {
  LLM_REQUIRE(g.M > 0 && g.N > 0 && g.K > 0 && (g.A || g.ln_x) && g.W_packed,
              "weight_gemm: bad arguments");
  LLM_REQUIRE(!g.ln_x || (g.ln_quant_only ? g.dtype == LLM_I8 && quant_prologue_ok(g.M, g.N, g.K)
                                           : g.ln_g && g.ln_b && ln_fusable(g.dtype, g.M, g.K)),
              "weight_gemm: LayerNorm / quantising prologue needs gamma / beta (LN) and an A "
              "image that fits LDS");
  const int kstep = g.dtype == LLM_I8 ? 64 : 32;
  LLM_REQUIRE(g.K % kstep == 0 && g.N % 16 == 0, "weight_gemm: K / N alignment");
  LLM_REQUIRE(g.a_packed || (g.lda >= g.K && g.lda % 16 == 0), "weight_gemm: lda");
  GemmArgs a{};
  a.A = static_cast<const uint8_t*>(g.A);
  a.lda = g.lda;
  a.a_packed = g.a_packed;
  a.B = static_cast<const uint8_t*>(g.W_packed);
  a.M = g.M; a.N = g.N; a.K = g.K; a.KS = g.K / kstep;
  a.sa = g.sa; a.sw = g.sw; a.bias = g.bias; a.act = g.act;
  a.C = g.C;
  a.c_cols = g.c_cols > 0 ? g.c_cols : g.N;
  a.c_ld = g.c_ld > 0 ? g.c_ld : g.N;
  LLM_REQUIRE(!g.C16 || g.N % 32 == 0, "weight_gemm: packed fp16 output needs N % 32 == 0");
  a.c16 = static_cast<_Float16*>(g.C16);
  a.ln_x = g.ln_x; a.ln_eps = g.ln_eps;
  a.ln_g = g.ln_quant_only ? nullptr : g.ln_g;
  a.ln_b = g.ln_quant_only ? nullptr : g.ln_b;
  a.ln_emb = g.ln_emb; a.ln_tok = g.ln_tok; a.ln_V = g.ln_V;
  a.act_out = static_cast<uint8_t*>(g.act_out);
  a.sa_out = g.sa_out;
  a.w_keep = g.w_keep;
  LLM_REQUIRE(!g.ksplit2 || (g.dtype == LLM_I8 && g.act == LLM_ACT_NONE && g.C && !g.C16 && !g.kv &&
                             !g.ln_x && (g.K / 64) >= 16 && (g.c_cols <= 0 || g.c_cols == g.N) &&
                             (g.c_ld <= 0 || g.c_ld >= g.N)),
              "weight_gemm: ksplit2 needs an I8 GEMM into all N columns of fp32 C with no "
              "activation, prologue, fp16 copy or KV append, and >= 16 k-steps");
  a.ksplit2 = g.ksplit2;
  if (g.kv) {
    const KvAppendView& kv = *g.kv;
    LLM_REQUIRE(g.N == 3 * kv.H * kv.D && g.K == kv.H * kv.D, "weight_gemm: kv append shape");
    a.kv = KvAppend{kv.pos, kv.page_table, kv.rows, static_cast<_Float16*>(kv.k_pool),
                    static_cast<_Float16*>(kv.v_pool), kv.num_beams, kv.max_tiles, kv.page_size,
                    kv.num_pages, kv.H, kv.D,
                    kv.page_stride > 0 ? kv.page_stride : (size_t)kv.page_size * kv.D};
  }
  const hipError_t e = g.dtype == LLM_I8 ? launch_gemm<GemmKind::I8>(a, st)
                                         : launch_gemm<GemmKind::F16>(a, st);
  if (e != hipSuccess) return fail(LLM_ERR_HIP, std::string("weight_gemm: ") + hipGetErrorString(e));
  return LLM_OK;
}
