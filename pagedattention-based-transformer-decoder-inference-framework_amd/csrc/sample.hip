// Device token sampling: temperature / top-k / top-p over
// the vocabulary, one workgroup per row, the row held in registers + LDS.
//
// Reference semantics restated:
//   * temperature + softmax: top_k_top_p_filter (attention/top_k_top_p_filter.cuh:55-88):
//       x_i = logit_i / T;  p_i = exp(x_i - max x) / (sum_j exp(x_j - max x) + 1e-6)
//   * filter: apply_topk_topp_filter (attention_cpu/softmax_lut.cpp:233-256): in
//     descending-probability order, token i is dropped when its rank >= top_k
//     (top_k > 0) or when the mass ranked above it has reached top_p
//     (top_p < 1); the two tests are independent.
//   * draw: the reference's device draw is `top_indices[rand() % top_k]`
//     (top_k_top_p_filter.cuh:107), which has no defined device RNG; this build
//     draws u ~ U[0,1) from a counter-based hash of (seed, row, counter) and takes
//     the inverse CDF of the kept mass in token-index order — deterministic and
//     replayable inside a hipGraph (the counter is device memory).
//   * greedy (T <= 0 or top_k == 1): argmax, first maximum wins
//     (sample_from_logits, decoder/cuda_decoder.cu:7-14).
//
// The rank / mass thresholds are found by a bitwise radix search over the
// (non-negative) fp32 probability bit patterns: 31 block-wide count or sum
// reductions per threshold, no sort.
#include "common.hpp"
#include "row_ops.hpp"

namespace llm {

constexpr int kSampleThreads = 512;  // 8 waves: 256 VGPRs per lane available

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [0, 1) with 24 random bits (exactly representable in fp32)
__host__ __device__ __forceinline__ float sample_uniform(uint64_t seed, int row, int counter) {
  uint64_t z = seed ^ ((uint64_t)(uint32_t)row << 32) ^ (uint64_t)(uint32_t)counter;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

struct SampleArgs {
  const float* logits;
  int V;
  float temperature;
  int top_k;
  float top_p;
  uint64_t seed;
  const int32_t* counter;  // per-row draw counter (device), or NULL -> counter0
  int counter0;
  int row0;                // row id of this launch's first row (for the draw)
  int32_t* out;
  int32_t* out2;  // optional second destination (stride out2_stride)
  int out2_stride;
};

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* sh, Op op) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = op(v, __shfl_xor(v, off, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  T t = sh[0];
  for (int i = 1; i < kSampleThreads / 64; ++i) t = op(t, sh[i]);  // fixed order
  return t;
}

// Thread t owns the contiguous tokens [t*VPT, t*VPT + VPT) of the row.  The
// first VPT_REG of them live in registers, the rest in LDS (VPT 128: 128 KiB,
// [slot][thread] so each access is bank-conflict free).
template <int VPT>
struct RowVals {
  // register slots; the rest in LDS: VPT 64 -> 32 + 64 KiB, VPT 128 -> 56 + 144 KiB
  static constexpr int R = VPT <= 32 ? VPT : (VPT <= 64 ? 32 : 56);
  float reg[R];
  // volatile: re-read per use, so the compiler does not hoist the LDS half into
  // registers across the radix-search loops (that spilled)
  volatile float* lds;  // [(VPT - R)][kSampleThreads]
  // f(i, value&): register slots unrolled, LDS slots in a rolled loop (dynamic
  // LDS indexing is free; unrolling it only made the compiler hoist and spill)
  template <typename F>
  __device__ __forceinline__ void each(F f) {
#pragma unroll
    for (int i = 0; i < R; ++i) f(i, reg[i]);
#pragma unroll 1
    for (int i = R; i < VPT; ++i) {
      float v = lds[(i - R) * kSampleThreads + threadIdx.x];
      f(i, v);
      lds[(i - R) * kSampleThreads + threadIdx.x] = v;
    }
  }
};

template <int VPT>
__global__ __launch_bounds__(kSampleThreads) void sample_rows_kernel(SampleArgs a) {
  __shared__ float shf[16];
  __shared__ int shi[16];
  __shared__ uint32_t shu[16];
  extern __shared__ float spill[];
  const int r = blockIdx.x;
  const float* lg = a.logits + (size_t)r * a.V;
  const int base = threadIdx.x * VPT;
  RowVals<VPT> p;
  p.lds = spill;
  const bool greedy = a.temperature <= 0.f || a.top_k == 1;
  p.each([&](int i, float& v) { v = base + i < a.V ? lg[base + i] : -INFINITY; });

  if (greedy) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    p.each([&](int i, float& v) {  // first max in the chunk
      if (v > best) { best = v; bi = base + i; }
    });
    const float m = block_reduce(best, shf, [](float x, float y) { return fmaxf(x, y); });
    int cand = (best == m) ? bi : 0x7fffffff;
    cand = block_reduce(cand, shi, [](int x, int y) { return min(x, y); });
    if (threadIdx.x == 0) {
      const int tok = cand == 0x7fffffff ? 0 : cand;
      a.out[r] = tok;
      if (a.out2) a.out2[(size_t)r * a.out2_stride] = tok;
    }
    return;
  }

  // temperature + softmax (reference: logits /= T; exp(x - max); / (sum + 1e-6))
  float mloc = -INFINITY;
  p.each([&](int, float& v) {
    v = v / a.temperature;
    mloc = fmaxf(mloc, v);
  });
  const float m = block_reduce(mloc, shf, [](float x, float y) { return fmaxf(x, y); });
  float sloc = 0.f;
  p.each([&](int i, float& v) {
    v = base + i < a.V ? expf(v - m) : 0.f;
    sloc += v;
  });
  const float s = block_reduce(sloc, shf, [](float x, float y) { return x + y; });
  const float inv = 1.0f / (s + 1e-6f);
  p.each([&](int, float& v) { v = v * inv; });

  // top-k: bit pattern of the k-th largest probability (keep bits >= tk)
  uint32_t tk = 0;
  if (a.top_k > 0 && a.top_k < a.V) {
    for (int bit = 30; bit >= 0; --bit) {
      const uint32_t cand = tk | (1u << bit);
      uint32_t c = 0;
      p.each([&](int, float& v) { c += __float_as_uint(v) >= cand; });
      c = block_reduce(c, shu, [](uint32_t x, uint32_t y) { return x + y; });
      if (c >= (uint32_t)a.top_k) tk = cand;
    }
  }
  // top-p: keep p_i iff the mass strictly above it is < top_p, i.e. bits > tp
  // where tp is the largest pattern whose strictly-above mass is >= top_p
  int64_t tp = -1;
  if (a.top_p < 1.0f) {
    auto mass_above = [&](uint32_t t) {
      float ms = 0.f;
      p.each([&](int, float& v) { ms += __float_as_uint(v) > t ? v : 0.f; });
      return block_reduce(ms, shf, [](float x, float y) { return x + y; });
    };
    if (mass_above(0u) >= a.top_p) {
      uint32_t t = 0;
      for (int bit = 30; bit >= 0; --bit) {
        const uint32_t cand = t | (1u << bit);
        if (mass_above(cand) >= a.top_p) t = cand;
      }
      tp = t;
    }
  }
  // kept mass in token-index order: thread partial sums, block exclusive scan
  float part = 0.f;
  p.each([&](int i, float& v) {
    const uint32_t bits = __float_as_uint(v);
    const bool keep = base + i < a.V && bits >= tk && (int64_t)bits > tp;
    v = keep ? v : 0.f;
    part += v;
  });
  __shared__ float scan[kSampleThreads];
  scan[threadIdx.x] = part;
  __syncthreads();
  for (int off = 1; off < kSampleThreads; off <<= 1) {  // Hillis-Steele inclusive scan
    const float v = threadIdx.x >= off ? scan[threadIdx.x - off] : 0.f;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  const float Z = scan[kSampleThreads - 1];
  const int ctr = a.counter ? a.counter[r] : a.counter0;
  const float target = sample_uniform(a.seed, a.row0 + r, ctr) * Z;
  const float lo = threadIdx.x ? scan[threadIdx.x - 1] : 0.f;
  // the thread whose [lo, lo + part) holds target picks inside its chunk
  int pick = 0x7fffffff;
  if (part > 0.f && target >= lo && (target < lo + part || threadIdx.x == kSampleThreads - 1 ||
                                     scan[threadIdx.x] >= Z)) {
    float c = lo;
    int last = -1;
    p.each([&](int i, float& v) {  // ascending token index
      if (v > 0.f) {
        last = base + i;
        c += v;
        if (target < c && pick == 0x7fffffff) pick = base + i;
      }
    });
    if (pick == 0x7fffffff) pick = last;  // rounding at the top of the range
  }
  pick = block_reduce(pick, shi, [](int x, int y) { return min(x, y); });
  if (threadIdx.x == 0) {
    const int tok = pick == 0x7fffffff ? 0 : pick;
    a.out[r] = tok;
    if (a.out2) a.out2[(size_t)r * a.out2_stride] = tok;
  }
}

template <int VPT>
hipError_t launch_sample_vpt(const SampleArgs& a, int rows, hipStream_t st) {
  constexpr size_t lds = (size_t)(VPT - RowVals<VPT>::R) * kSampleThreads * sizeof(float);
  if constexpr (lds > 65536) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sample_rows_kernel<VPT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
  }
  hipLaunchKernelGGL(sample_rows_kernel<VPT>, dim3(rows), dim3(kSampleThreads), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_sample_rows(const SampleArgs& a, int rows, hipStream_t st) {
  const int vpt = (a.V + kSampleThreads - 1) / kSampleThreads;
  if (vpt <= 16) return launch_sample_vpt<16>(a, rows, st);
  if (vpt <= 32) return launch_sample_vpt<32>(a, rows, st);
  if (vpt <= 64) return launch_sample_vpt<64>(a, rows, st);
  if (vpt <= 128) return launch_sample_vpt<128>(a, rows, st);
  return hipErrorInvalidValue;
}

}  // namespace llm

using namespace llm;

extern "C" int sample_rows(const float* logits, int rows, int V, float temperature, int top_k,
                           float top_p, uint64_t seed, int counter, int32_t* out, void* stream) {
  LLM_REQUIRE(rows >= 0 && V > 0, "sample_rows: bad shape");
  if (rows == 0) return LLM_OK;
  LLM_REQUIRE(logits && out, "sample_rows: NULL pointer");
  LLM_REQUIRE(V <= 128 * kSampleThreads, "sample_rows: V > 65536");
  LLM_REQUIRE(top_k >= 0 && top_p > 0.f && top_p <= 1.0f, "sample_rows: top_k >= 0, 0 < top_p <= 1");
  SampleArgs a{logits, V, temperature, top_k, top_p, seed, nullptr, counter, 0, out, nullptr, 0};
  LLM_HIP_RET(launch_sample_rows(a, rows, as_stream(stream)));
  return LLM_OK;
}

hipError_t llm::launch_sample(const float* logits, int rows, int row0, int V, float temperature,
                              int top_k, float top_p, uint64_t seed, const int32_t* counter,
                              int32_t* out, hipStream_t st) {
  SampleArgs a{logits, V, temperature, top_k, top_p, seed, counter, 0, row0, out, nullptr, 0};
  return launch_sample_rows(a, rows, st);
}

extern "C" float sample_uniform_host(uint64_t seed, int row, int counter) {
  return sample_uniform(seed, row, counter);
}
