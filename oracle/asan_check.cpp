// ORACLE — TEST INFRASTRUCTURE ONLY.  AddressSanitizer / UBSan run of the CPU
// restatement (sanitizer build of the CPU path): drives every
// oracle entry point at small, ragged shapes — missing pages, page ids past the
// pool, beam routing, ragged contexts, filters, the decoder step with and
// without teacher forcing — so an out-of-bounds read or write in the checker
// fails here instead of silently corrupting a parity verdict.
//   make -C oracle asan   (builds ../oracle/_asan/asan_check and runs it)
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

extern "C" {
int oracle_paged_attention(const float*, const float*, const float*, const int32_t*, int, int, int,
                           int, const int32_t*, const int32_t*, int, int, int, int, float, int,
                           float, int, float, float*, float*, float*);
void oracle_quantize_rows(const float*, int, int, int8_t*, float*);
void oracle_quantize_cols(const float*, int, int, int8_t*, float*);
void oracle_i8_gemm(const int8_t*, const int8_t*, int32_t*, float*, int, int, int, const float*,
                    const float*, const float*, int);
void oracle_layer_norm(const float*, int, int, const float*, const float*, float, float*);
void oracle_mlp_f32(const float*, int, int, int, const float*, const float*, const float*,
                    const float*, float*);
void oracle_argmax_rows(const float*, int, int, int32_t*);
struct oracle_model {
  int L, H, D, hid, inter, V, max_seq;
  const uint16_t* emb;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  const int8_t* wqkv; const float* sw_qkv;
  const int8_t* wo;   const float* sw_o;
  const int8_t* w1;   const float* sw1; const float* b1;
  const int8_t* w2;   const float* sw2; const float* b2;
  const uint16_t *hwqkv, *hwo, *hw1, *hw2;
};
void* oracle_decoder_create(const oracle_model*, int);
void oracle_decoder_destroy(void*);
int oracle_decoder_step(void*, const int32_t*, const int32_t*, float, int, int, float*, float*,
                        int32_t*);
int oracle_decoder_step_forced(void*, const int32_t*, const int32_t*, float, float*, int32_t*,
                               const int8_t*, const float*, float*);
}

template <typename T>
static std::vector<T> randn(std::mt19937& g, size_t n, float s) {
  std::normal_distribution<float> d(0.f, s);
  std::vector<T> v(n);
  for (auto& x : v) x = (T)d(g);
  return v;
}

int main() {
  std::mt19937 g(7);
  int fails = 0;
  // paged attention: ts 16, ragged T, missing pages, an out-of-pool id, beam routing
  for (int D : {32, 64, 128}) {
    const int B = 3, H = 2, ts = 16, T = 70, beams = 2, nt = (T + ts - 1) / ts, pages = beams * H * nt;
    auto q = randn<float>(g, (size_t)B * H * D, 0.3f);
    auto k = randn<float>(g, (size_t)pages * ts * D, 0.3f), v = randn<float>(g, (size_t)pages * ts * D, 1.f);
    std::vector<int32_t> pt((size_t)beams * H * nt);
    for (size_t i = 0; i < pt.size(); ++i) pt[i] = (int32_t)((i * 7) % pages);
    pt[1] = -1;
    pt[3] = pages + 5;  // past the pool: treated as missing
    std::vector<int32_t> bid = {1, 0, 1}, ctx = {70, 33, 1};
    std::vector<float> out((size_t)B * H * D), pr((size_t)B * H * T), sc((size_t)B * H * T);
    fails += oracle_paged_attention(q.data(), k.data(), v.data(), pt.data(), pages, ts, beams, nt,
                                    bid.data(), ctx.data(), B, H, D, T, 1.f, 0, 1.f, -1, 0.f,
                                    out.data(), pr.data(), sc.data()) != 0;
    fails += oracle_paged_attention(q.data(), k.data(), v.data(), pt.data(), pages, ts, beams, nt,
                                    bid.data(), nullptr, B, H, D, T, 0.7f, 5, 0.9f, 3, 1e-3f,
                                    out.data(), pr.data(), sc.data()) != 0;
  }
  // GEMM, quantisers, LayerNorm, MLP, argmax at ragged sizes
  {
    const int M = 5, K = 192, N = 40;
    auto a = randn<float>(g, (size_t)M * K, 1.f), w = randn<float>(g, (size_t)K * N, 0.05f);
    std::vector<int8_t> qa((size_t)M * K), qw((size_t)K * N);
    std::vector<float> sa(M), sw(N), c((size_t)M * N), bias = randn<float>(g, N, 0.1f);
    std::vector<int32_t> acc((size_t)M * N), am(M);
    oracle_quantize_rows(a.data(), M, K, qa.data(), sa.data());
    oracle_quantize_cols(w.data(), K, N, qw.data(), sw.data());
    for (int act = 0; act < 3; ++act)
      oracle_i8_gemm(qa.data(), qw.data(), acc.data(), c.data(), M, N, K, sa.data(), sw.data(),
                     bias.data(), act);
    auto gm = randn<float>(g, K, 1.f), bt = randn<float>(g, K, 0.1f);
    std::vector<float> ln((size_t)M * K);
    oracle_layer_norm(a.data(), M, K, gm.data(), bt.data(), 1e-5f, ln.data());
    auto w1 = randn<float>(g, (size_t)K * 4 * K, 0.05f), b1 = randn<float>(g, 4 * K, 0.05f);
    auto w2 = randn<float>(g, (size_t)4 * K * K, 0.05f), b2 = randn<float>(g, K, 0.05f);
    std::vector<float> mo((size_t)M * K);
    oracle_mlp_f32(a.data(), M, K, 4 * K, w1.data(), b1.data(), w2.data(), b2.data(), mo.data());
    oracle_argmax_rows(c.data(), M, N, am.data());
  }
  // decoder step: 2 layers, ragged positions, forced and free
  {
    const int L = 2, H = 2, D = 64, hid = H * D, inter = 4 * hid, V = 97, S = 24, B = 3;
    std::vector<uint16_t> emb((size_t)V * hid, 0x3400);
    auto ones = std::vector<float>((size_t)L * hid, 1.f), zeros = std::vector<float>((size_t)L * hid, 0.f);
    std::vector<int8_t> wqkv((size_t)L * hid * 3 * hid, 3), wo((size_t)L * hid * hid, -2),
        w1((size_t)L * hid * inter, 1), w2((size_t)L * inter * hid, -1);
    std::vector<float> s3((size_t)L * 3 * hid, 1e-3f), s1((size_t)L * hid, 1e-3f),
        si((size_t)L * inter, 1e-3f), bi((size_t)L * inter, 0.01f);
    oracle_model m{L, H, D, hid, inter, V, S, emb.data(), ones.data(), zeros.data(), ones.data(),
                   zeros.data(), wqkv.data(), s3.data(), wo.data(), s1.data(), w1.data(), si.data(),
                   bi.data(), w2.data(), s1.data(), zeros.data(), nullptr, nullptr, nullptr,
                   nullptr};
    void* d = oracle_decoder_create(&m, B);
    std::vector<float> x((size_t)B * hid), lg((size_t)B * V), st((size_t)L * 12);
    std::vector<int32_t> nx(B);
    std::vector<int8_t> fq((size_t)L * 4 * B * inter, 1);
    std::vector<float> fs((size_t)L * 4 * B, 1e-2f);
    for (int s = 0; s < 4; ++s) {
      std::vector<int32_t> tok = {s, 2 * s + 1, 96}, pos = {s, s + 5, S - 4 + s};
      fails += oracle_decoder_step(d, tok.data(), pos.data(), 1.f, -1, 1, x.data(), lg.data(), nx.data()) != 0;
      fails += oracle_decoder_step_forced(d, tok.data(), pos.data(), 1.f, lg.data(), nx.data(),
                                          fq.data(), fs.data(), st.data()) != 0;
    }
    std::vector<int32_t> bad = {0, 0, V}, pos = {0, 0, 0};
    fails += oracle_decoder_step(d, bad.data(), pos.data(), 1.f, -1, 1, nullptr, nullptr, nullptr) == 0;
    oracle_decoder_destroy(d);
    // the CUDADecoder (fp16 weights) restatement
    std::vector<uint16_t> hq((size_t)L * hid * 3 * hid, 0x2000), ho((size_t)L * hid * hid, 0xA000),
        h1w((size_t)L * hid * inter, 0x2000), h2w((size_t)L * inter * hid, 0xA000);
    m.hwqkv = hq.data(); m.hwo = ho.data(); m.hw1 = h1w.data(); m.hw2 = h2w.data();
    d = oracle_decoder_create(&m, B);
    for (int s = 0; s < 3; ++s) {
      std::vector<int32_t> tok = {s, 5, 96}, p2 = {s, s + 2, S - 3 + s};
      fails += oracle_decoder_step(d, tok.data(), p2.data(), 1.f, -1, 1, x.data(), lg.data(), nx.data()) != 0;
    }
    fails += oracle_decoder_step_forced(d, bad.data(), pos.data(), 1.f, lg.data(), nx.data(),
                                        fq.data(), fs.data(), st.data()) == 0;
    oracle_decoder_destroy(d);
  }
  std::printf("asan_check: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
