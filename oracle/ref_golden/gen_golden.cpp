// Golden-vector generator — TEST INFRASTRUCTURE ONLY (runs in the build
// container, never on the GPU box, never shipped).
//
// Links the reference's own compilable sources, where they lie under
// /root/reference (see Makefile in this directory):
//   kv_cache/kv_tile_cache_cpu.cpp   KVTileCacheCPU<float|uint16_t|int8_t>  (put/get/save/load)
//   attention_cpu/softmax_lut.cpp    softmax_lut_vec, apply_topk_topp_filter
//   attention_cpu/int8_quant.cpp     quantize_to_int8, batch_quantize, ...
//   decoder/layer_norm.hpp, decoder/mlp.hpp, decoder/token_embedding.hpp (header-only)
// and drives them the way cpu_paged_attention_forward
// (attention_cpu/cpu_attention_kernel.cpp:37-129) does; that function itself
// does not compile, so its loop is re-driven here with the
// reference's cache, softmax and filter.  Inputs/outputs are raw little-endian
// files in a scratch directory; tests/golden/make_golden.py packs them into the
// committed fixtures.

#include "kv_cache/kv_tile_cache_cpu.hpp"
#include "attention_cpu/softmax_lut.hpp"
#include "attention_cpu/int8_quant.hpp"
#include "decoder/layer_norm.hpp"
#include "decoder/mlp.hpp"
#include "decoder/token_embedding.hpp"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

template <typename T>
static std::vector<T> read_file(const std::string& path, size_t n) {
  std::vector<T> v(n);
  std::ifstream f(path, std::ios::binary);
  if (!f) { std::fprintf(stderr, "cannot open %s\n", path.c_str()); std::exit(2); }
  f.read(reinterpret_cast<char*>(v.data()), n * sizeof(T));
  if (!f) { std::fprintf(stderr, "short read %s\n", path.c_str()); std::exit(2); }
  return v;
}

template <typename T>
static void write_file(const std::string& path, const T* p, size_t n) {
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(p), n * sizeof(T));
}

// attn <dir> B H D T ts beams temperature top_k top_p eos eos_thr has_beam_ids
static int run_attn(int argc, char** argv) {
  if (argc < 15) return 1;
  const std::string dir = argv[2];
  const int B = atoi(argv[3]), H = atoi(argv[4]), D = atoi(argv[5]), T = atoi(argv[6]);
  const int ts = atoi(argv[7]), beams = atoi(argv[8]);
  const float temperature = (float)atof(argv[9]);
  const int top_k = atoi(argv[10]);
  const float top_p = (float)atof(argv[11]);
  const int eos = atoi(argv[12]);
  const float eos_thr = (float)atof(argv[13]);
  const int has_beam_ids = atoi(argv[14]);
  const int nt = (T + ts - 1) / ts;

  auto q = read_file<float>(dir + "/q.f32", (size_t)B * H * D);
  auto k = read_file<float>(dir + "/k.f32", (size_t)beams * H * nt * ts * D);
  auto v = read_file<float>(dir + "/v.f32", (size_t)beams * H * nt * ts * D);
  auto present = read_file<int32_t>(dir + "/present.i32", (size_t)beams * H * nt);
  std::vector<int32_t> beam_ids;
  if (has_beam_ids) beam_ids = read_file<int32_t>(dir + "/beam_ids.i32", B);

  // Two caches: KVTileCacheCPU's tile_size_ counts ELEMENTS (kv_tile_cache_cpu.cpp:33,41),
  // so one tile of ts tokens x D dims has tile_size_ = ts * D.
  KVTileCacheCPU<float> kc(beams * H * nt + 1, ts * D), vc(beams * H * nt + 1, ts * D);
  for (int r = 0; r < beams; ++r)
    for (int h = 0; h < H; ++h)
      for (int t = 0; t < nt; ++t) {
        const size_t ti = ((size_t)r * H + h) * nt + t;
        if (!present[ti]) continue;
        kc.put(r, h, t, k.data() + ti * ts * D);
        vc.put(r, h, t, v.data() + ti * ts * D);
      }

  std::vector<float> out((size_t)B * H * D, 0.f), probs_all((size_t)B * H * T), scores_all((size_t)B * H * T);
  for (int b = 0; b < B; ++b) {
    for (int h = 0; h < H; ++h) {
      const int beam = has_beam_ids ? beam_ids[b] : b;             // :50
      const float* qv = q.data() + ((size_t)b * H + h) * D;
      std::vector<float> scores(T, -1e9f), probs(T, 0.0f);         // :61
      for (int tile = 0; tile < nt; ++tile) {                      // :68-86
        const int start = tile * ts;
        const int len = std::min(ts, T - start);
        const float* kt = kc.get(beam, h, tile);
        if (!kt) continue;
        for (int t = 0; t < len; ++t) {
          float dot = 0.0f;
          for (int d = 0; d < D; ++d) dot += qv[d] * kt[t * D + d];
          scores[start + t] = dot / temperature;                   // :85 (causal=false)
        }
      }
      softmax_lut_vec(scores.data(), T, temperature, probs.data()); // :90
      apply_topk_topp_filter(probs.data(), T, top_k, top_p, eos, eos_thr);  // :93-97
      float* o = out.data() + ((size_t)b * H + h) * D;
      for (int tile = 0; tile < nt; ++tile) {                      // :103-117
        const int start = tile * ts;
        const int len = std::min(ts, T - start);
        const float* vt = vc.get(beam, h, tile);
        if (!vt) continue;
        for (int t = 0; t < len; ++t)
          for (int d = 0; d < D; ++d) o[d] += probs[start + t] * vt[t * D + d];
      }
      std::copy(probs.begin(), probs.end(), probs_all.begin() + ((size_t)b * H + h) * T);
      std::copy(scores.begin(), scores.end(), scores_all.begin() + ((size_t)b * H + h) * T);
    }
  }
  write_file(dir + "/out.f32", out.data(), out.size());
  write_file(dir + "/probs.f32", probs_all.data(), probs_all.size());
  write_file(dir + "/scores.f32", scores_all.data(), scores_all.size());
  return 0;
}

// softmax <dir> len temperature
static int run_softmax(int argc, char** argv) {
  if (argc < 5) return 1;
  const std::string dir = argv[2];
  const int len = atoi(argv[3]);
  const float temperature = (float)atof(argv[4]);
  auto s = read_file<float>(dir + "/scores.f32", len);
  std::vector<float> out(len);
  softmax_lut_vec(s.data(), len, temperature, out.data());
  write_file(dir + "/out.f32", out.data(), out.size());
  return 0;
}

// quant <dir> n rows   (x: [rows][n/rows])
static int run_quant(int argc, char** argv) {
  if (argc < 5) return 1;
  const std::string dir = argv[2];
  const int n = atoi(argv[3]), rows = atoi(argv[4]);
  auto x = read_file<float>(dir + "/x.f32", n);
  const float scale = compute_minmax_scale(x);
  auto q = quantize_to_int8(x, scale);
  auto dq = dequantize_from_int8(q, scale);
  const float absmax = compute_absmax(x);
  // per-row (batch_quantize with per-row minmax scales)
  const int dim = n / rows;
  std::vector<float> scales(rows);
  for (int r = 0; r < rows; ++r) {
    std::vector<float> row(x.begin() + (size_t)r * dim, x.begin() + (size_t)(r + 1) * dim);
    scales[r] = compute_minmax_scale(row);
  }
  auto qr = batch_quantize(x, scales, dim);
  auto dqr = batch_dequantize(qr, scales, dim);
  write_file(dir + "/scale.f32", &scale, 1);
  write_file(dir + "/absmax.f32", &absmax, 1);
  write_file(dir + "/q.i8", q.data(), q.size());
  write_file(dir + "/dq.f32", dq.data(), dq.size());
  write_file(dir + "/row_scales.f32", scales.data(), scales.size());
  write_file(dir + "/qr.i8", qr.data(), qr.size());
  write_file(dir + "/dqr.f32", dqr.data(), dqr.size());
  return 0;
}

// ln <dir> rows cols
static int run_ln(int argc, char** argv) {
  if (argc < 5) return 1;
  const std::string dir = argv[2];
  const int rows = atoi(argv[3]), cols = atoi(argv[4]);
  auto x = read_file<float>(dir + "/x.f32", (size_t)rows * cols);
  LayerNorm<float> ln(cols);
  ln.load_weights(dir + "/gamma_beta.f32");  // gamma then beta (layer_norm.hpp:13-18)
  std::vector<float> out((size_t)rows * cols);
  ln.forward(x.data(), out.data(), rows);
  write_file(dir + "/out.f32", out.data(), out.size());
  return 0;
}

// mlp <dir> rows hid inter
static int run_mlp(int argc, char** argv) {
  if (argc < 6) return 1;
  const std::string dir = argv[2];
  const int rows = atoi(argv[3]), hid = atoi(argv[4]), inter = atoi(argv[5]);
  auto x = read_file<float>(dir + "/x.f32", (size_t)rows * hid);
  MLP<float> mlp(hid, inter);
  mlp.load_weights(dir + "/mlp.f32");  // fc1_w, fc1_b, fc2_w, fc2_b (mlp.hpp:14-21)
  std::vector<float> out((size_t)rows * hid);
  mlp.forward(x.data(), out.data(), rows);
  write_file(dir + "/out.f32", out.data(), out.size());
  return 0;
}

// embed <dir> vocab hid n_ids
static int run_embed(int argc, char** argv) {
  if (argc < 6) return 1;
  const std::string dir = argv[2];
  const int vocab = atoi(argv[3]), hid = atoi(argv[4]), n = atoi(argv[5]);
  auto ids = read_file<int32_t>(dir + "/ids.i32", n);
  TokenEmbedding<float> emb(vocab, hid);
  emb.load_weights(dir + "/emb.f32");
  std::vector<int> idv(ids.begin(), ids.end());
  std::vector<float> out;
  emb.forward(idv, out);
  write_file(dir + "/out.f32", out.data(), out.size());
  return 0;
}

// KVTileCacheCPU<T>::save / load (kv_cache/kv_tile_cache_cpu.cpp:89-123): the
// reference's on-disk tile-record format.  Inputs: idx.i32 [n][3] (batch, head,
// tile) and data.bin (n tiles of tile_elems elements of T, raw bits).  The
// reference's save() writes tiles.bin; a second cache load()s it and get()s
// every index back into back.bin, so the fixture pins both directions.
template <typename T>
static int kvtiles_t(const std::string& dir, int n, int tile_elems) {
  auto idx = read_file<int32_t>(dir + "/idx.i32", (size_t)n * 3);
  auto data = read_file<T>(dir + "/data.bin", (size_t)n * tile_elems);
  KVTileCacheCPU<T> c(n + 1, tile_elems);
  for (int i = 0; i < n; ++i)
    c.put(idx[3 * i], idx[3 * i + 1], idx[3 * i + 2], data.data() + (size_t)i * tile_elems);
  c.save(dir + "/tiles.bin");
  KVTileCacheCPU<T> r(n + 1, tile_elems);
  r.load(dir + "/tiles.bin");
  std::vector<T> back((size_t)n * tile_elems);
  for (int i = 0; i < n; ++i) {
    const T* t = r.get(idx[3 * i], idx[3 * i + 1], idx[3 * i + 2]);
    if (!t) { std::fprintf(stderr, "record %d lost in load\n", i); return 3; }
    std::copy(t, t + tile_elems, back.begin() + (size_t)i * tile_elems);
  }
  write_file(dir + "/back.bin", back.data(), back.size());
  return 0;
}

// kvtiles <dir> n tile_elems elem_bytes(1|2|4)
static int run_kvtiles(int argc, char** argv) {
  if (argc < 6) return 1;
  const std::string dir = argv[2];
  const int n = atoi(argv[3]), te = atoi(argv[4]), es = atoi(argv[5]);
  if (es == 1) return kvtiles_t<int8_t>(dir, n, te);
  if (es == 2) return kvtiles_t<uint16_t>(dir, n, te);
  if (es == 4) return kvtiles_t<float>(dir, n, te);
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: gen_golden <attn|softmax|quant|ln|mlp|embed|kvtiles> ...\n"); return 1; }
  const std::string cmd = argv[1];
  if (cmd == "attn") return run_attn(argc, argv);
  if (cmd == "softmax") return run_softmax(argc, argv);
  if (cmd == "quant") return run_quant(argc, argv);
  if (cmd == "ln") return run_ln(argc, argv);
  if (cmd == "mlp") return run_mlp(argc, argv);
  if (cmd == "embed") return run_embed(argc, argv);
  if (cmd == "kvtiles") return run_kvtiles(argc, argv);
  return 1;
}
