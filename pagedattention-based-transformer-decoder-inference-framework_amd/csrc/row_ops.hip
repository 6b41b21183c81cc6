// Row-wise decoder glue kernels: LayerNorm (+ fused int8 quantisation),
// per-row int8 quantisation, embedding gather, KV append into pages, argmax.
// All are one workgroup per row, vectorised 16 B per lane where the row allows.
#include "common.hpp"
#include "gemm.hpp"
#include "ln_wave.hpp"
#include "row_ops.hpp"

namespace llm {

constexpr int kRowThreads = 256;

__device__ __forceinline__ float block_reduce_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) t += sh[i];  // fixed order: deterministic
  return t;
}

__device__ __forceinline__ float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float t = sh[0];
  const int nw = blockDim.x >> 6;
  for (int i = 1; i < nw; ++i) t = fmaxf(t, sh[i]);
  return t;
}

// int8_quant.cpp:5-13,59-64: scale = 127/(absmax + 1e-6), q = clamp(round(x*scale)).
__device__ __forceinline__ int8_t quant1(float x, float scale) {
  float y = roundf(__fmul_rn(x, scale));
  y = fminf(fmaxf(y, -128.f), 127.f);
  return (int8_t)(int)y;
}

// Quantise one row held by the block (values in `vals`, VPT per thread,
// element index i = threadIdx.x + k*blockDim.x).
__global__ __launch_bounds__(kRowThreads) void quantize_rows_kernel(const float* __restrict__ x,
                                                                    int cols, int8_t* __restrict__ q,
                                                                    float* __restrict__ inv_scale) {
  __shared__ float sh[kRowThreads / 64];
  const int r = blockIdx.x;
  const float* xr = x + (size_t)r * cols;
  float am = 0.f;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) am = fmaxf(am, fabsf(xr[i]));
  am = block_reduce_max(am, sh);
  const float scale = 127.f / (am + 1e-6f);
  int8_t* qr = q + (size_t)r * cols;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) qr[i] = quant1(xr[i], scale);
  if (threadIdx.x == 0) inv_scale[r] = 1.0f / scale;
}

// LayerNorm<T>::forward (decoder/layer_norm.hpp:20-37): biased variance,
// inv_std = 1.0/sqrt(var + eps), out = (x - mean) * inv_std * gamma + beta
// (left-to-right, not contracted), then optional per-row int8 quantisation.
__global__ __launch_bounds__(kRowThreads) void layernorm_quant_kernel(
    const float* __restrict__ x, int cols, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ out, int8_t* __restrict__ q,
    float* __restrict__ inv_scale, _Float16* __restrict__ out16) {
  extern __shared__ __attribute__((aligned(16))) float row[];  // cols floats
  __shared__ float sh[kRowThreads / 64];
  const int r = blockIdx.x;
  const float* xr = x + (size_t)r * cols;
  float s = 0.f;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) {
    const float v = xr[i];
    row[i] = v;
    s += v;
  }
  const float mean = block_reduce_sum(s, sh) / (float)cols;
  float vs = 0.f;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) {
    const float d = row[i] - mean;
    vs = fmaf(d, d, vs);
  }
  const float var = block_reduce_sum(vs, sh) / (float)cols;
  const float inv_std = (float)(1.0 / (double)sqrtf(var + eps));
  float am = 0.f;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) {
    float y = __fmul_rn(__fmul_rn(row[i] - mean, inv_std), gamma[i]);
    y = __fadd_rn(y, beta[i]);
    row[i] = y;
    am = fmaxf(am, fabsf(y));
    if (out) out[(size_t)r * cols + i] = y;
    if (out16) out16[(size_t)r * cols + i] = (_Float16)y;
  }
  if (q) {
    am = block_reduce_max(am, sh);
    const float scale = 127.f / (am + 1e-6f);
    for (int i = threadIdx.x; i < cols; i += blockDim.x) q[(size_t)r * cols + i] = quant1(row[i], scale);
    if (threadIdx.x == 0) inv_scale[r] = 1.0f / scale;
  }
}

// ---------------------------------------------------------------------------
// Register-resident row kernels (cols % 4 == 0, cols <= 1024 * VPT): every
// thread loads its VPT float4 chunks of the row (chunk i = threadIdx.x + 256 v)
// with all loads in flight at once, so a row costs ONE memory round trip; the
// reductions are wave DPP/shuffles + one LDS exchange; int8 results leave as
// one packed dword per float4.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float block_sum_fast(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();  // sh reuse across consecutive reductions
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);  // fixed order: deterministic
}

__device__ __forceinline__ float block_max_fast(float v, float* sh) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

__device__ __forceinline__ uint32_t pack4_i8(f32x4 y, float scale) {
  const uint32_t b0 = (uint8_t)quant1(y[0], scale), b1 = (uint8_t)quant1(y[1], scale);
  const uint32_t b2 = (uint8_t)quant1(y[2], scale), b3 = (uint8_t)quant1(y[3], scale);
  return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

// pack = 1: q / out16 are written in packed-A order (a_frag_off_*), else row-major.
template <int VPT>
__global__ __launch_bounds__(kRowThreads) void quantize_rows_v_kernel(
    const float* __restrict__ x, int cols, int8_t* __restrict__ q, float* __restrict__ inv_scale,
    int pack) {
  __shared__ float sh[4];
  const int r = blockIdx.x;
  const int n4 = cols >> 2;
  const f32x4* xr = reinterpret_cast<const f32x4*>(x + (size_t)r * cols);
  f32x4 v[VPT];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kRowThreads;
    v[i] = c < n4 ? xr[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i)
    am = fmaxf(am, fmaxf(fmaxf(fabsf(v[i][0]), fabsf(v[i][1])), fmaxf(fabsf(v[i][2]), fabsf(v[i][3]))));
  am = block_max_fast(am, sh);
  const float scale = 127.f / (am + 1e-6f);
  uint32_t* qr = reinterpret_cast<uint32_t*>(q + (size_t)r * cols);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kRowThreads;
    if (c < n4) {
      if (pack)
        *reinterpret_cast<uint32_t*>(q + a_frag_off_i8(r, 4 * c, cols >> 6)) = pack4_i8(v[i], scale);
      else
        qr[c] = pack4_i8(v[i], scale);
    }
  }
  if (threadIdx.x == 0) inv_scale[r] = 1.0f / scale;
}

// LayerNorm (+ int8 quantisation) launch, one 256-thread workgroup per row:
// every thread loads its VPT float4 chunks (chunk c = threadIdx.x + 256 v) of
// x (or of the embedding row E[tok[r]], pp.emb) and gamma / beta, all in ONE
// memory round trip;
// wave DPP sums + one LDS exchange per reduction.  Numerics of
// LayerNorm<T>::forward (decoder/layer_norm.hpp:20-37) and int8_quant.cpp as
// ln_wave.hpp (the GEMM prologue); only the fp32 summation order differs.
// q / out16 in packed-A order when pack.
template <int VPT>
__global__ __launch_bounds__(kRowThreads) void layernorm_rows_kernel(
    const float* x /* not restrict: pp.zero_x may point at it (fc2_split) */, int rows, int cols, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ out, int8_t* __restrict__ q,
    float* __restrict__ inv_scale, _Float16* __restrict__ out16, int pack, LnSource pp) {
  __shared__ float sh[4];
  const int r = blockIdx.x;
  const int n4 = cols >> 2;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(gamma);
  const f32x4* b4 = reinterpret_cast<const f32x4*>(beta);
  f32x4 v[VPT], gv[VPT], bv[VPT];
  if (pp.emb) {  // x = E[tok[r]] (embed_kernel's values, not stored)
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4* er = reinterpret_cast<const h4*>(ln_embed_row(pp.emb, pp.tok, r, pp.V, cols));
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kRowThreads;
      const bool ok = c < n4;
      const h4 e = ok ? er[c] : h4{0, 0, 0, 0};
      v[i] = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
      gv[i] = ok ? g4[c] : f32x4{0.f, 0.f, 0.f, 0.f};
      bv[i] = ok ? b4[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
    const f32x4* xr = reinterpret_cast<const f32x4*>(x + (size_t)r * cols);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kRowThreads;
      const bool ok = c < n4;
      v[i] = ok ? xr[c] : f32x4{0.f, 0.f, 0.f, 0.f};
      gv[i] = ok ? g4[c] : f32x4{0.f, 0.f, 0.f, 0.f};
      bv[i] = ok ? b4[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  const float mean = block_sum_fast(s, sh) / (float)cols;
  if (pp.zero_x && !pp.emb) {  // (after the barrier in block_sum_fast: every thread's loads are done)
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kRowThreads;
      if (c < n4) reinterpret_cast<f32x4*>(pp.zero_x + (size_t)r * cols)[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float vs = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kRowThreads;
    if (c < n4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[i][e] - mean;
        vs = fmaf(d, d, vs);
      }
    }
  }
  const float var = block_sum_fast(vs, sh) / (float)cols;
  const float inv_std = (float)(1.0 / (double)sqrtf(var + eps));
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float y = __fmul_rn(__fmul_rn(v[i][e] - mean, inv_std), gv[i][e]);
      v[i][e] = __fadd_rn(y, bv[i][e]);
      am = fmaxf(am, fabsf(v[i][e]));  // padding chunks: beta 0 -> 0
    }
  }
  const float scale = q ? 127.f / (block_max_fast(am, sh) + 1e-6f) : 1.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kRowThreads;
    if (c >= n4) continue;
    const int k = 4 * c;
    if (out) reinterpret_cast<f32x4*>(out + (size_t)r * cols)[c] = v[i];
    if (q)
      *reinterpret_cast<uint32_t*>(q + (pack ? a_frag_off_i8(r, k, cols >> 6) : (size_t)r * cols + k)) =
          ln_quant4(v[i], scale);
    if (out16)
      *reinterpret_cast<ln_f16x4*>(out16 + (pack ? a_frag_off_f16(r, k, cols >> 5) : (size_t)r * cols + k)) =
          ln_half4(v[i]);
  }
  if (q && threadIdx.x == 0) inv_scale[r] = 1.0f / scale;
}

// VPT (float4 chunks per thread) for a row of `cols`; 0 = use the scalar kernel.
static int row_vpt(int cols) {
  if (cols % 4 != 0) return 0;
  const int n4 = cols / 4;
  for (int v : {1, 2, 4, 8, 16})
    if (n4 <= v * kRowThreads) return v;
  return 0;
}

// Argmax per row, first maximum wins (std::max_element).
__global__ __launch_bounds__(kRowThreads) void argmax_kernel(const float* __restrict__ logits,
                                                             int V, int32_t* __restrict__ out,
                                                             int32_t* __restrict__ out2,
                                                             int out2_stride) {
  __shared__ float shv[kRowThreads];
  __shared__ int shi[kRowThreads];
  const int r = blockIdx.x;
  const float* l = logits + (size_t)r * V;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = l[i];
    if (v > best) { best = v; bi = i; }  // strided scan: first index per thread
  }
  shv[threadIdx.x] = best;
  shi[threadIdx.x] = bi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const float v2 = shv[threadIdx.x + s];
      const int i2 = shi[threadIdx.x + s];
      if (v2 > shv[threadIdx.x] || (v2 == shv[threadIdx.x] && i2 < shi[threadIdx.x])) {
        shv[threadIdx.x] = v2;
        shi[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int idx = shi[0] == 0x7fffffff ? 0 : shi[0];
    out[r] = idx;
    if (out2) out2[(size_t)r * out2_stride] = idx;
  }
}

// x[b] = float(E[tok[b]]) (TokenEmbedding::forward, decoder/token_embedding.hpp:19-26).
__global__ __launch_bounds__(kRowThreads) void embed_kernel(const _Float16* __restrict__ E,
                                                            const int32_t* __restrict__ tok,
                                                            int hid, int V,
                                                            float* __restrict__ x) {
  const int b = blockIdx.x;
  int t = tok[b];
  t = t < 0 ? 0 : (t >= V ? V - 1 : t);
  const _Float16* e = E + (size_t)t * hid;
  float* xr = x + (size_t)b * hid;
  for (int i = threadIdx.x; i < hid; i += blockDim.x) xr[i] = (float)e[i];
}

// pack_cols > 0: y is packed-A fp16 of rows of pack_cols (x row-major [n / pack_cols][pack_cols]).
__global__ void to_f16_kernel(const float* __restrict__ x, size_t n, _Float16* __restrict__ y,
                              int pack_cols) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    if (pack_cols > 0) {
      const int m = (int)(i / pack_cols), k = (int)(i % pack_cols);
      y[a_frag_off_f16(m, k, pack_cols >> 5)] = (_Float16)x[i];
    } else {
      y[i] = (_Float16)x[i];
    }
  }
}

// After a step: every row's next position / context length moves by one.
__global__ void advance_kernel(int32_t* __restrict__ pos, int32_t* __restrict__ ctx, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    pos[i] += 1;
    ctx[i] += 1;
  }
}

// page_table[idx[i]] = val[i] (device half of PageTable sync).
__global__ void scatter_i32_kernel(int32_t* __restrict__ dst, const int64_t* __restrict__ idx,
                                   const int32_t* __restrict__ val, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = val[i];
}

// Seeded random fp16 fill (synthetic KV contexts): splitmix64 -> ~N(0,1)*scale
// via the sum of 4 uniforms (Irwin-Hall), cheap and deterministic.
// Element i of the n = pages * page_elems lands at p[(i / page_elems) *
// page_stride + i % page_elems] (page_stride in elements: a pool whose pages
// interleave with another pool's).
__global__ void fill_random_f16_kernel(_Float16* __restrict__ p, size_t n, size_t page_elems,
                                       size_t page_stride, uint64_t seed, float scale) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    float u = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) u += (float)((z >> (16 * k)) & 0xFFFF) * (1.0f / 65536.0f);
    p[(i / page_elems) * page_stride + i % page_elems] = (_Float16)((u - 2.0f) * 1.7320508f * scale);
  }
}

// ---------------------------------------------------------------------------
// host launchers (internal)
// ---------------------------------------------------------------------------
hipError_t launch_quantize_rows(const float* x, int rows, int cols, int8_t* q, float* inv,
                                hipStream_t st, int pack) {
  const dim3 g(rows), b(kRowThreads);
  const int v = row_vpt(cols);
  if (pack && (v == 0 || cols % 64 != 0)) return hipErrorInvalidValue;
  switch (v) {
    case 1: hipLaunchKernelGGL(quantize_rows_v_kernel<1>, g, b, 0, st, x, cols, q, inv, pack); break;
    case 2: hipLaunchKernelGGL(quantize_rows_v_kernel<2>, g, b, 0, st, x, cols, q, inv, pack); break;
    case 4: hipLaunchKernelGGL(quantize_rows_v_kernel<4>, g, b, 0, st, x, cols, q, inv, pack); break;
    case 8: hipLaunchKernelGGL(quantize_rows_v_kernel<8>, g, b, 0, st, x, cols, q, inv, pack); break;
    case 16: hipLaunchKernelGGL(quantize_rows_v_kernel<16>, g, b, 0, st, x, cols, q, inv, pack); break;
    default: hipLaunchKernelGGL(quantize_rows_kernel, g, b, 0, st, x, cols, q, inv); break;
  }
  return hipGetLastError();
}

static hipError_t launch_ln(const float* x, int rows, int cols, const float* g, const float* b,
                            float eps, float* out, int8_t* q, float* inv, _Float16* out16,
                            hipStream_t st, int pack, const LnSource* pp = nullptr) {
  const LnSource none{};
  const int v = row_vpt(cols);
  if (pack && (v == 0 || cols % 64 != 0)) return hipErrorInvalidValue;
  if (pp && pp->emb && v == 0) return hipErrorInvalidValue;
  if (v == 0) {  // odd widths (C ABI only)
    hipLaunchKernelGGL(layernorm_quant_kernel, dim3(rows), dim3(kRowThreads),
                       (size_t)cols * sizeof(float), st, x, cols, g, b, eps, out, q, inv, out16);
    return hipGetLastError();
  }
  const dim3 gr(rows), bl(kRowThreads);
#define LN_CASE(V)                                                                              \
  if (v == V) {                                                                                 \
    hipLaunchKernelGGL((layernorm_rows_kernel<V>), gr, bl, 0, st, x, rows, cols, g, b, eps, out, \
                       q, inv, out16, pack, pp ? *pp : none);                                   \
    return hipGetLastError();                                                                   \
  }
  LN_CASE(1) LN_CASE(2) LN_CASE(4) LN_CASE(8) LN_CASE(16)
#undef LN_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_layernorm_quant(const float* x, int rows, int cols, const float* g,
                                  const float* b, float eps, float* out, int8_t* q, float* inv,
                                  hipStream_t st, int pack, const LnSource* pp) {
  return launch_ln(x, rows, cols, g, b, eps, out, q, inv, nullptr, st, pack, pp);
}

hipError_t launch_layernorm_f16(const float* x, int rows, int cols, const float* g,
                                const float* b, float eps, void* out16, hipStream_t st, int pack,
                                const LnSource* pp) {
  return launch_ln(x, rows, cols, g, b, eps, nullptr, nullptr, nullptr,
                   static_cast<_Float16*>(out16), st, pack, pp);
}

hipError_t launch_to_f16(const float* x, size_t n, void* y, hipStream_t st, int pack_cols) {
  if (n == 0) return hipSuccess;
  if (pack_cols > 0 && pack_cols % 32 != 0) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(to_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n,
                     static_cast<_Float16*>(y), pack_cols);
  return hipGetLastError();
}

hipError_t launch_advance(int32_t* pos, int32_t* ctx, int n, hipStream_t st) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(256), 0, st, pos, ctx, n);
  return hipGetLastError();
}

hipError_t launch_argmax(const float* logits, int rows, int V, int32_t* out, int32_t* out2,
                         int out2_stride, hipStream_t st) {
  hipLaunchKernelGGL(argmax_kernel, dim3(rows), dim3(kRowThreads), 0, st, logits, V, out, out2,
                     out2_stride);
  return hipGetLastError();
}

hipError_t launch_embed(const void* E, const int32_t* tok, int rows, int hid, int V, float* x,
                        hipStream_t st) {
  hipLaunchKernelGGL(embed_kernel, dim3(rows), dim3(kRowThreads), 0, st,
                     static_cast<const _Float16*>(E), tok, hid, V, x);
  return hipGetLastError();
}

hipError_t launch_scatter_i32(int32_t* dst, const int64_t* idx, const int32_t* val, int n,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_i32_kernel, dim3((n + 255) / 256), dim3(256), 0, st, dst, idx, val, n);
  return hipGetLastError();
}

hipError_t launch_fill_random_f16(void* p, size_t pages, size_t page_elems, size_t page_stride,
                                  uint64_t seed, float scale, hipStream_t st) {
  const size_t n = pages * page_elems;
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(fill_random_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     static_cast<_Float16*>(p), n, page_elems, page_stride, seed, scale);
  return hipGetLastError();
}

}  // namespace llm

using namespace llm;

extern "C" int quantize_rows(const float* x, int rows, int cols, int8_t* q, float* inv_scale,
                             void* stream) {
  LLM_REQUIRE(rows >= 0 && cols > 0, "quantize_rows: bad shape");
  if (rows == 0) return LLM_OK;
  LLM_REQUIRE(x && q && inv_scale, "quantize_rows: NULL pointer");
  LLM_HIP_RET(launch_quantize_rows(x, rows, cols, q, inv_scale, as_stream(stream), 0));
  return LLM_OK;
}

extern "C" int layernorm_quant(const float* x, int rows, int cols, const float* gamma,
                               const float* beta, float eps, float* out, int8_t* q,
                               float* inv_scale, void* stream) {
  LLM_REQUIRE(rows >= 0 && cols > 0, "layernorm_quant: bad shape");
  if (rows == 0) return LLM_OK;
  LLM_REQUIRE(x && gamma && beta, "layernorm_quant: NULL pointer");
  LLM_REQUIRE((q == nullptr) == (inv_scale == nullptr), "layernorm_quant: q and inv_scale go together");
  LLM_REQUIRE(out || q, "layernorm_quant: no output requested");
  LLM_REQUIRE(cols <= 16384, "layernorm_quant: cols > 16384 (LDS row buffer)");
  LLM_HIP_RET(launch_layernorm_quant(x, rows, cols, gamma, beta, eps, out, q, inv_scale,
                                     as_stream(stream), 0));
  return LLM_OK;
}

extern "C" int argmax_rows(const float* logits, int rows, int V, int32_t* out, void* stream) {
  LLM_REQUIRE(rows >= 0 && V > 0, "argmax_rows: bad shape");
  if (rows == 0) return LLM_OK;
  LLM_REQUIRE(logits && out, "argmax_rows: NULL pointer");
  LLM_HIP_RET(launch_argmax(logits, rows, V, out, nullptr, 0, as_stream(stream)));
  return LLM_OK;
}
