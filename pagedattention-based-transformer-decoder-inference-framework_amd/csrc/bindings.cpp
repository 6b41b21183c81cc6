// pybind11 module `llm_decoder` — the reference's Python surface
// (src/bindings.cpp:3-35, include/bindings.hpp:1-10) over the C ABI of
// libllm_decoder_hip.so (include/llm_decoder.h).
//
//   CUDADecoder(num_layers, num_heads, head_dim, hidden_dim, vocab_size, max_seq_len)
//       .load_weights(path) / .generate(...)                       bindings.cpp:5-15
//   INT8Decoder(same)
//       .load_quantized_weights(path) / .quantize_weights(src, dst) / .generate(...)
//                                                                  bindings.cpp:18-29
// generate accepts both call conventions in the tree:
//   generate(input_ids, max_len, temperature=1.0) -> list           (bindings.cpp:8-15)
//   generate(input_ids, output_ids, max_gen_len, temperature=1.0)   (api/router.py:23,
//       web/app.py:23, cli/chat_cli.py:24 — fills output_ids in place)
// and both return / fill prompt + generated ids (cuda_decoder.cu:49,59).
// Additions: generate_batch, set_weights (host numpy arrays), low-level
// begin_synthetic / step for the bench, PageTable / KVTileCache classes with
// the kv_cache/ API names (page_table.hpp:5-37, kv_tile_cache.hpp:9-41) and
// paged_attention() over raw device pointers.
//
// Errors: any non-zero C-ABI status raises RuntimeError with llm_last_error().
// The GIL is released around device work; each decoder serialises its own
// calls with an internal mutex (KVTileCache's std::mutex, kv_tile_cache.hpp:73).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "llm_decoder.h"

namespace py = pybind11;

namespace {

void check(int rc) {
  if (rc != LLM_OK) throw std::runtime_error(std::string("llm_decoder: ") + llm_last_error());
}

template <typename T>
py::array_t<T, py::array::c_style | py::array::forcecast> arr(const py::dict& w, const char* k,
                                                                size_t expect) {
  if (!w.contains(k)) throw std::invalid_argument(std::string("set_weights: missing '") + k + "'");
  auto a = py::array_t<T, py::array::c_style | py::array::forcecast>::ensure(w[k]);
  if (!a) throw std::invalid_argument(std::string("set_weights: bad array '") + k + "'");
  if ((size_t)a.size() != expect)
    throw std::invalid_argument(std::string("set_weights: '") + k + "' has " +
                                std::to_string(a.size()) + " elements, expected " +
                                std::to_string(expect));
  return a;
}

class Decoder {
 public:
  Decoder(int weight_dtype, int num_layers, int num_heads, int head_dim, int hidden_dim,
          int vocab_size, int max_seq_len, int max_batch, int page_size, int inter_dim,
          float attn_scale, long long num_pages) {
    llm_decoder_config c{};
    c.num_layers = num_layers; c.num_heads = num_heads; c.head_dim = head_dim;
    c.hidden_dim = hidden_dim; c.vocab_size = vocab_size; c.max_seq_len = max_seq_len;
    c.inter_dim = inter_dim; c.page_size = page_size; c.weight_dtype = weight_dtype;
    c.max_batch = max_batch; c.attn_scale = attn_scale; c.num_pages = num_pages;
    check(llm_decoder_create(&c, &d_));
    cfg_ = c;
    if (cfg_.inter_dim <= 0) cfg_.inter_dim = 4 * hidden_dim;
  }
  ~Decoder() { llm_decoder_destroy(d_); }
  Decoder(const Decoder&) = delete;
  Decoder& operator=(const Decoder&) = delete;

  void load_weights(const std::string& path) {
    py::gil_scoped_release nogil;
    check(llm_decoder_load_weights(d_, path.c_str()));
  }
  void load_quantized_weights(const std::string& path) {
    py::gil_scoped_release nogil;
    check(llm_decoder_load_quantized_weights(d_, path.c_str()));
  }
  void quantize_weights(const std::string& src, const std::string& dst) {
    py::gil_scoped_release nogil;
    check(llm_quantize_weights(src.c_str(), dst.c_str(), cfg_.num_layers, cfg_.hidden_dim,
                               cfg_.inter_dim, cfg_.vocab_size));
  }

  void set_weights(const py::dict& w) {
    const size_t L = cfg_.num_layers, hid = cfg_.hidden_dim, inter = cfg_.inter_dim,
                 V = cfg_.vocab_size;
    auto emb = arr<uint16_t>(w, "emb", V * hid);
    auto ln1_g = arr<float>(w, "ln1_g", L * hid), ln1_b = arr<float>(w, "ln1_b", L * hid);
    auto ln2_g = arr<float>(w, "ln2_g", L * hid), ln2_b = arr<float>(w, "ln2_b", L * hid);
    auto b1 = arr<float>(w, "b1", L * inter), b2 = arr<float>(w, "b2", L * hid);
    if (cfg_.weight_dtype == LLM_I8) {
      auto wqkv = arr<int8_t>(w, "wqkv", L * hid * 3 * hid), wo = arr<int8_t>(w, "wo", L * hid * hid);
      auto w1 = arr<int8_t>(w, "w1", L * hid * inter), w2 = arr<int8_t>(w, "w2", L * inter * hid);
      auto sq = arr<float>(w, "sw_qkv", L * 3 * hid), so = arr<float>(w, "sw_o", L * hid);
      auto s1 = arr<float>(w, "sw1", L * inter), s2 = arr<float>(w, "sw2", L * hid);
      llm_int8_weights x{emb.data(), ln1_g.data(), ln1_b.data(), ln2_g.data(), ln2_b.data(),
                         wqkv.data(), sq.data(), wo.data(), so.data(), w1.data(), s1.data(),
                         b1.data(), w2.data(), s2.data(), b2.data()};
      py::gil_scoped_release nogil;
      check(llm_decoder_set_int8_weights(d_, &x));
    } else {
      auto wqkv = arr<uint16_t>(w, "wqkv", L * hid * 3 * hid), wo = arr<uint16_t>(w, "wo", L * hid * hid);
      auto w1 = arr<uint16_t>(w, "w1", L * hid * inter), w2 = arr<uint16_t>(w, "w2", L * inter * hid);
      llm_f16_weights x{emb.data(), ln1_g.data(), ln1_b.data(), ln2_g.data(), ln2_b.data(),
                        wqkv.data(), wo.data(), w1.data(), w2.data(), b1.data(), b2.data()};
      py::gil_scoped_release nogil;
      check(llm_decoder_set_f16_weights(d_, &x));
    }
  }

  std::vector<std::vector<int>> generate_batch(const std::vector<std::vector<int>>& prompts,
                                               int max_gen_len, float temperature) {
    const int B = (int)prompts.size();
    if (B == 0) return {};
    size_t stride = 1;
    for (auto& p : prompts) stride = std::max(stride, p.size());
    std::vector<int32_t> flat((size_t)B * stride, 0), lens(B);
    for (int b = 0; b < B; ++b) {
      lens[b] = (int32_t)prompts[b].size();
      std::copy(prompts[b].begin(), prompts[b].end(), flat.begin() + (size_t)b * stride);
    }
    std::vector<int32_t> out((size_t)B * std::max(max_gen_len, 0));
    {
      py::gil_scoped_release nogil;
      check(llm_decoder_generate(d_, flat.data(), lens.data(), (int)stride, B, max_gen_len,
                                 temperature, out.data()));
    }
    std::vector<std::vector<int>> res(B);
    for (int b = 0; b < B; ++b) {
      res[b] = prompts[b];  // output_ids = input_ids (cuda_decoder.cu:49)
      for (int g = 0; g < max_gen_len; ++g) res[b].push_back(out[(size_t)b * max_gen_len + g]);
    }
    return res;
  }

  py::object generate(py::args args, py::kwargs kwargs) {
    // form 1: (input_ids, max_len[, temperature]) -> list
    // form 2: (input_ids, output_ids: list, max_gen_len[, temperature]) -> None
    std::vector<int> input;
    py::object out_list = py::none();
    int max_len = -1;
    float temperature = 1.0f;
    size_t i = 0;
    if (args.size() > i) input = args[i++].cast<std::vector<int>>();
    else if (kwargs.contains("input_ids")) input = kwargs["input_ids"].cast<std::vector<int>>();
    else throw std::invalid_argument("generate: input_ids is required");
    if (args.size() > i && py::isinstance<py::list>(args[i])) out_list = args[i++];
    else if (kwargs.contains("output_ids")) out_list = kwargs["output_ids"];
    if (args.size() > i) max_len = args[i++].cast<int>();
    for (const char* k : {"max_gen_len", "max_len", "max_tokens"})
      if (kwargs.contains(k)) max_len = kwargs[k].cast<int>();
    if (args.size() > i) temperature = args[i++].cast<float>();
    if (kwargs.contains("temperature")) temperature = kwargs["temperature"].cast<float>();
    if (max_len < 0) throw std::invalid_argument("generate: max_gen_len is required");
    if (input.empty()) throw std::invalid_argument("generate: input_ids must not be empty");
    auto res = generate_batch({input}, max_len, temperature)[0];
    if (!out_list.is_none()) {
      py::list l = out_list.cast<py::list>();
      while (py::len(l) > 0) l.attr("pop")();
      for (int t : res) l.append(t);
      return py::none();
    }
    return py::cast(res);
  }

  void begin_synthetic(int batch, int context_len, uint64_t seed, bool shuffle) {
    py::gil_scoped_release nogil;
    check(llm_decoder_begin_synthetic(d_, batch, context_len, seed, shuffle ? 1 : 0));
  }

  void prefill(int row, const std::vector<int32_t>& tokens) {
    py::gil_scoped_release nogil;
    check(llm_decoder_prefill(d_, row, tokens.data(), (int)tokens.size()));
  }

  void set_sampling(float temperature, int top_k, float top_p, uint64_t seed) {
    py::gil_scoped_release nogil;
    check(llm_decoder_set_sampling(d_, temperature, top_k, top_p, seed));
  }

  void begin_beams(int num_seqs, int beam_width, int shared_len, int beam_len, uint64_t seed,
                   bool shuffle) {
    py::gil_scoped_release nogil;
    check(llm_decoder_begin_beams(d_, num_seqs, beam_width, shared_len, beam_len, seed,
                                  shuffle ? 1 : 0));
  }

  py::object step(py::object tokens, uintptr_t logits_ptr, uintptr_t stream, bool want_next) {
    std::vector<int32_t> tok;
    const int32_t* tp = nullptr;
    if (!tokens.is_none()) {
      tok = tokens.cast<std::vector<int32_t>>();
      tp = tok.data();
    }
    int n = 0;
    for (;; ++n)
      if (llm_decoder_context_len(d_, n) < 0) break;
    if (tp && (int)tok.size() != n) throw std::invalid_argument("step: need one token per active row");
    std::vector<int32_t> next(want_next ? n : 0);
    {
      py::gil_scoped_release nogil;
      check(llm_decoder_step(d_, tp, reinterpret_cast<float*>(logits_ptr),
                             want_next ? next.data() : nullptr, reinterpret_cast<void*>(stream)));
    }
    if (!want_next) return py::none();
    return py::cast(std::vector<int>(next.begin(), next.end()));
  }

  void sync() {
    py::gil_scoped_release nogil;
    check(llm_decoder_sync(d_));
  }
  void copy_next_ids(uintptr_t dst, uintptr_t stream) {
    py::gil_scoped_release nogil;
    check(llm_decoder_copy_next(d_, reinterpret_cast<int32_t*>(dst), reinterpret_cast<void*>(stream)));
  }
  // llm_decoder_set_taps: device pointers (0, 0 switches the taps off)
  void set_taps(uintptr_t q_ptr, uintptr_t s_ptr) {
    py::gil_scoped_release nogil;
    check(llm_decoder_set_taps(d_, reinterpret_cast<int8_t*>(q_ptr), reinterpret_cast<float*>(s_ptr)));
  }
  int context_len(int row) const { return llm_decoder_context_len(d_, row); }
  void run_attention(int layer, uintptr_t stream) {
    py::gil_scoped_release nogil;
    check(llm_decoder_run_attention(d_, layer, reinterpret_cast<void*>(stream)));
  }
  // llm_decoder_oproj_status: (range guard tripped, accumulator columns not at zero)
  py::tuple oproj_status() {
    int clamped = 0;
    long long nz = 0;
    {
      py::gil_scoped_release nogil;
      check(llm_decoder_oproj_status(d_, &clamped, &nz));
    }
    return py::make_tuple(clamped != 0, nz);
  }
  // llm_decoder_attention_plan: (splits per (row, head), LLM_PA_FORM_*)
  py::tuple attention_plan() {
    int ns = 0, form = 0;
    check(llm_decoder_attention_plan(d_, &ns, &form));
    return py::make_tuple(ns, form);
  }
  uintptr_t kv_handle() const { return reinterpret_cast<uintptr_t>(llm_decoder_kv(d_)); }
  const llm_decoder_config& config() const { return cfg_; }

 private:
  llm_decoder* d_ = nullptr;
  llm_decoder_config cfg_{};
};

class CUDADecoder : public Decoder {
 public:
  CUDADecoder(int L, int H, int D, int hid, int V, int S, int max_batch, int page_size, int inter,
              float attn_scale, long long num_pages)
      : Decoder(LLM_F16, L, H, D, hid, V, S, max_batch, page_size, inter, attn_scale, num_pages) {}
};

class INT8Decoder : public Decoder {
 public:
  INT8Decoder(int L, int H, int D, int hid, int V, int S, int max_batch, int page_size, int inter,
              float attn_scale, long long num_pages)
      : Decoder(LLM_I8, L, H, D, hid, V, S, max_batch, page_size, inter, attn_scale, num_pages) {}
};

// KVTileCache<T> (kv_cache/kv_tile_cache.hpp:9-41) with a layer dimension.
class KVTileCache {
 public:
  KVTileCache() = default;
  ~KVTileCache() { if (c_) kv_cache_destroy(c_); }
  // dtype: the T of KVTileCache<T> — "float16" (default), "bfloat16", "float32", "int8"
  void init(int num_pages, int tile_size, int head_dim, int num_layers, int num_beams,
            int num_heads, int max_tiles, const std::string& dtype) {
    const int kvt = dtype == "float16" || dtype == "half" ? LLM_F16
                    : dtype == "bfloat16"                 ? LLM_BF16
                    : dtype == "float32" || dtype == "float" ? LLM_F32
                    : dtype == "int8"                     ? LLM_I8
                                                          : -1;
    if (kvt < 0) throw std::invalid_argument("KVTileCache: dtype must be float16, bfloat16, float32 or int8");
    if (c_) { kv_cache_destroy(c_); c_ = nullptr; }
    check(kv_cache_create_typed(num_layers, num_beams, num_heads, head_dim, tile_size, max_tiles,
                                num_pages, kvt, &c_));
    tile_size_ = tile_size; head_dim_ = head_dim; layers_ = num_layers; beams_ = num_beams;
    heads_ = num_heads; max_tiles_ = max_tiles; dtype_ = dtype;
    es_ = kvt == LLM_F32 ? 4 : kvt == LLM_I8 ? 1 : 2;
  }
  void resize(int new_num_pages, int new_tile_size) {  // kv_tile_cache.cpp:26-37: drops contents
    init(new_num_pages, new_tile_size, head_dim_, layers_, beams_, heads_, max_tiles_, dtype_);
  }
  uintptr_t get_key_ptr(int page) const {
    need();
    if (page < 0 || page >= kv_cache_num_pages(c_)) throw std::out_of_range("page id");
    return reinterpret_cast<uintptr_t>(kv_cache_k_pool(c_)) + (uintptr_t)page * kv_cache_page_stride(c_);
  }
  uintptr_t get_value_ptr(int page) const {
    need();
    if (page < 0 || page >= kv_cache_num_pages(c_)) throw std::out_of_range("page id");
    return reinterpret_cast<uintptr_t>(kv_cache_v_pool(c_)) + (uintptr_t)page * kv_cache_page_stride(c_);
  }
  int register_tile(int beam, int head, int tile, int layer) {
    need();
    int32_t page = -1;
    check(kv_cache_register_tile(c_, layer, beam, head, tile, &page));
    return page;
  }
  int lookup(int beam, int head, int tile, int layer) const {
    need();
    return kv_cache_lookup(c_, layer, beam, head, tile);
  }
  // "lru": KVTileCache's eviction when the pool is full (kv_tile_cache.cpp:89-98);
  // "none" (default): register_tile raises instead
  void set_eviction(const std::string& policy) {
    need();
    if (policy != "lru" && policy != "none")
      throw std::invalid_argument("KVTileCache.set_eviction: policy must be 'lru' or 'none'");
    check(kv_cache_set_eviction(c_, policy == "lru" ? LLM_EVICT_LRU : LLM_EVICT_NONE));
  }
  void fork(int src, int dst) { need(); check(kv_cache_fork(c_, src, dst)); }
  void release(int beam) { need(); check(kv_cache_release(c_, beam)); }
  void sync_page_table_to_gpu() { need(); check(kv_cache_sync(c_, nullptr)); check(llm_sync()); }
  // KVTileCache::save_to_file / load_from_file (kv_tile_cache.cpp:105-125):
  // format "pools" (default) is the reference's file byte for byte (raw K pool
  // then V pool; the page table stays as it is); "snapshot" is this build's
  // file that also restores the layered page table.
  void save_to_file(const std::string& p, const std::string& format) {
    need();
    check(fmt(format) ? kv_cache_save(c_, p.c_str()) : kv_cache_save_pools(c_, p.c_str()));
  }
  void load_from_file(const std::string& p, const std::string& format) {
    need();
    check(fmt(format) ? kv_cache_load(c_, p.c_str()) : kv_cache_load_pools(c_, p.c_str()));
  }
  // KVTileCacheCPU<T>::save / load (kv_tile_cache_cpu.cpp:89-123): the K ("k")
  // or V ("v") tiles of one layer as the reference's record file
  void save_tiles(const std::string& p, const std::string& kind, int layer) {
    need();
    check(kv_cache_save_tiles(c_, layer, kind_of(kind), p.c_str()));
  }
  void load_tiles(const std::string& p, const std::string& kind, int layer) {
    need();
    check(kv_cache_load_tiles(c_, layer, kind_of(kind), p.c_str()));
  }
  // k / v: C-contiguous [n][H][D] arrays whose items are the cache's element
  // bits (fp16/bf16 as uint16 or float16, float32, int8).
  void write_tokens(int layer, int beam, int pos, py::array k, py::array v) {
    need();
    const bool contig = (k.flags() & py::array::c_style) && (v.flags() & py::array::c_style);
    if (!contig || k.itemsize() != es_ || v.itemsize() != es_ || k.size() != v.size() ||
        k.size() % ((size_t)heads_ * head_dim_) != 0)
      throw std::invalid_argument("write_tokens: k/v must be C-contiguous [n][H][D] arrays of the "
                                  "cache's element size");
    const int n = (int)(k.size() / ((size_t)heads_ * head_dim_));
    check(kv_cache_write_tokens(c_, layer, beam, pos, n, k.data(), v.data()));
  }
  py::dict view(int layer) const {
    need();
    pa_kv_view v;
    check(kv_cache_view(c_, layer, &v));
    py::dict d;
    d["k_pool"] = reinterpret_cast<uintptr_t>(v.k_pool);
    d["v_pool"] = reinterpret_cast<uintptr_t>(v.v_pool);
    d["page_table"] = reinterpret_cast<uintptr_t>(v.page_table);
    d["num_pages"] = v.num_pages; d["page_size"] = v.page_size; d["head_dim"] = v.head_dim;
    d["num_beams"] = v.num_beams; d["num_heads"] = v.num_heads; d["max_tiles"] = v.max_tiles;
    d["kv_dtype"] = v.kv_dtype;
    d["page_stride"] = v.page_stride;
    return d;
  }
  long long free_pages() const { need(); return kv_cache_free_pages(c_); }
  long long num_pages() const { need(); return kv_cache_num_pages(c_); }
  uintptr_t handle() const { return reinterpret_cast<uintptr_t>(c_); }

 private:
  static int llm_sync() { return LLM_OK; }
  static bool fmt(const std::string& f) {
    if (f == "pools") return false;
    if (f == "snapshot") return true;
    throw std::invalid_argument("KVTileCache: format must be 'pools' (the reference's file) or 'snapshot'");
  }
  static int kind_of(const std::string& k) {
    if (k == "k" || k == "K") return 0;
    if (k == "v" || k == "V") return 1;
    throw std::invalid_argument("KVTileCache: kind must be 'k' or 'v'");
  }
  void need() const { if (!c_) throw std::runtime_error("KVTileCache: call init() first"); }
  kv_cache* c_ = nullptr;
  int tile_size_ = 0, head_dim_ = 0, layers_ = 1, beams_ = 1, heads_ = 1, max_tiles_ = 1;
  int es_ = 2;
  std::string dtype_ = "float16";
};

// PageTable (kv_cache/page_table.hpp:5-37): a one-layer table whose entries
// name pages of an external pool; backed by a kv_cache with 1-element pages.
class PageTable {
 public:
  PageTable() = default;
  ~PageTable() { if (c_) kv_cache_destroy(c_); }
  void init(int num_beams, int num_heads, int num_tiles) {
    if (c_) { kv_cache_destroy(c_); c_ = nullptr; }
    const long long pages = std::max<long long>(1, (long long)num_beams * num_heads * num_tiles);
    check(kv_cache_create(1, num_beams, num_heads, 1, 1, num_tiles, pages, &c_));
  }
  void clear() { need(); check(kv_cache_clear(c_)); }
  void assign(int beam, int head, int tile, int page) {
    need();
    check(kv_cache_assign(c_, 0, beam, head, tile, page));
    check(kv_cache_sync(c_, nullptr));
  }
  int lookup(int beam, int head, int tile) const { need(); return kv_cache_lookup(c_, 0, beam, head, tile); }
  void remove(int beam, int head, int tile) { need(); check(kv_cache_remove(c_, 0, beam, head, tile)); }
  void sync_to_gpu() { need(); check(kv_cache_sync(c_, nullptr)); }
  uintptr_t device_data() const { need(); return reinterpret_cast<uintptr_t>(kv_cache_page_table(c_, 0)); }

 private:
  void need() const { if (!c_) throw std::runtime_error("PageTable: call init() first"); }
  kv_cache* c_ = nullptr;
};

}  // namespace

PYBIND11_MODULE(llm_decoder, m) {
  m.doc() = "MI355X (gfx950) paged-attention decoder: CUDADecoder / INT8Decoder (HIP)";
  m.attr("ABI_VERSION") = llm_abi_version();

  auto dec_init = [](auto* cls) {
    return py::init([](int L, int H, int D, int hid, int V, int S, int max_batch, int page_size,
                       int inter, float attn_scale, long long num_pages) {
             return new std::remove_pointer_t<decltype(cls)>(L, H, D, hid, V, S, max_batch,
                                                             page_size, inter, attn_scale,
                                                             num_pages);
           });
  };
  auto common = [&](auto& c) {
    c.def("load_weights", &Decoder::load_weights, "CUDADecoder::load_weights (fp32 .bin dir)")
        .def("set_weights", &Decoder::set_weights, py::arg("weights"))
        .def("generate", &Decoder::generate)
        .def("generate_batch", &Decoder::generate_batch, py::arg("input_ids"),
             py::arg("max_gen_len"), py::arg("temperature") = 1.0f)
        .def("begin_synthetic", &Decoder::begin_synthetic, py::arg("batch"),
             py::arg("context_len"), py::arg("seed") = 0, py::arg("shuffle") = true)
        .def("prefill", &Decoder::prefill, py::arg("row"), py::arg("tokens"))
        .def("set_sampling", &Decoder::set_sampling, py::arg("temperature"),
             py::arg("top_k") = 0, py::arg("top_p") = 1.0f, py::arg("seed") = 0)
        .def("begin_beams", &Decoder::begin_beams, py::arg("num_seqs"), py::arg("beam_width"),
             py::arg("shared_len"), py::arg("beam_len"), py::arg("seed") = 0,
             py::arg("shuffle") = true)
        .def("step", &Decoder::step, py::arg("tokens") = py::none(), py::arg("logits_ptr") = 0,
             py::arg("stream") = 0, py::arg("want_next") = true)
        .def("sync", &Decoder::sync)
        .def("set_taps", &Decoder::set_taps, py::arg("q_ptr"), py::arg("s_ptr"))
        .def("copy_next_ids", &Decoder::copy_next_ids, py::arg("dst_ptr"), py::arg("stream") = 0)
        .def("context_len", &Decoder::context_len)
        .def("attention_plan", &Decoder::attention_plan)
        .def("oproj_status", &Decoder::oproj_status)
        .def("run_attention", &Decoder::run_attention, py::arg("layer") = 0,
             py::arg("stream") = 0)
        .def_property_readonly("kv_handle", &Decoder::kv_handle);
  };
  py::class_<Decoder>(m, "_Decoder");
  py::class_<CUDADecoder, Decoder> cd(m, "CUDADecoder");
  cd.def(dec_init((CUDADecoder*)nullptr), py::arg("num_layers"), py::arg("num_heads"),
         py::arg("head_dim"), py::arg("hidden_dim"), py::arg("vocab_size"),
         py::arg("max_seq_len"), py::arg("max_batch") = 1, py::arg("page_size") = 16,
         py::arg("inter_dim") = 0, py::arg("attn_scale") = 1.0f, py::arg("num_pages") = 0);
  common(cd);
  py::class_<INT8Decoder, Decoder> id(m, "INT8Decoder");
  id.def(dec_init((INT8Decoder*)nullptr), py::arg("num_layers"), py::arg("num_heads"),
         py::arg("head_dim"), py::arg("hidden_dim"), py::arg("vocab_size"),
         py::arg("max_seq_len"), py::arg("max_batch") = 1, py::arg("page_size") = 16,
         py::arg("inter_dim") = 0, py::arg("attn_scale") = 1.0f, py::arg("num_pages") = 0);
  common(id);
  id.def("load_quantized_weights", &Decoder::load_quantized_weights)
      .def("quantize_weights", &Decoder::quantize_weights);

  py::class_<KVTileCache>(m, "KVTileCache")
      .def(py::init<>())
      .def("init", &KVTileCache::init, py::arg("num_pages"), py::arg("tile_size"),
           py::arg("head_dim"), py::arg("num_layers") = 1, py::arg("num_beams") = 1,
           py::arg("num_heads") = 1, py::arg("max_tiles") = 1, py::arg("dtype") = "float16")
      .def("resize", &KVTileCache::resize)
      .def("get_key_ptr", &KVTileCache::get_key_ptr)
      .def("get_value_ptr", &KVTileCache::get_value_ptr)
      .def("register_tile", &KVTileCache::register_tile, py::arg("beam_id"), py::arg("head_id"),
           py::arg("tile_id"), py::arg("layer") = 0)
      .def("lookup", &KVTileCache::lookup, py::arg("beam_id"), py::arg("head_id"),
           py::arg("tile_id"), py::arg("layer") = 0)
      .def("set_eviction", &KVTileCache::set_eviction, py::arg("policy"))
      .def("fork", &KVTileCache::fork)
      .def("release", &KVTileCache::release)
      .def("sync_page_table_to_gpu", &KVTileCache::sync_page_table_to_gpu)
      .def("save_to_file", &KVTileCache::save_to_file, py::arg("path"),
           py::arg("format") = "pools")
      .def("load_from_file", &KVTileCache::load_from_file, py::arg("path"),
           py::arg("format") = "pools")
      .def("save_tiles", &KVTileCache::save_tiles, py::arg("path"), py::arg("kind") = "k",
           py::arg("layer") = 0)
      .def("load_tiles", &KVTileCache::load_tiles, py::arg("path"), py::arg("kind") = "k",
           py::arg("layer") = 0)
      .def("write_tokens", &KVTileCache::write_tokens)
      .def("view", &KVTileCache::view, py::arg("layer") = 0)
      .def("free_pages", &KVTileCache::free_pages)
      .def("num_pages", &KVTileCache::num_pages)
      .def_property_readonly("handle", &KVTileCache::handle);

  py::class_<PageTable>(m, "PageTable")
      .def(py::init<>())
      .def("init", &PageTable::init)
      .def("clear", &PageTable::clear)
      .def("assign", &PageTable::assign)
      .def("lookup", &PageTable::lookup)
      .def("remove", &PageTable::remove)
      .def("sync_to_gpu", &PageTable::sync_to_gpu)
      .def("device_data", &PageTable::device_data);

  m.def("paged_attention",
        [](uintptr_t kv_handle, int layer, uintptr_t q, uintptr_t out, uintptr_t beam_ids,
           uintptr_t context_lens, int B, int H, int D, int T, float temperature, int top_k,
           float top_p, uintptr_t workspace, size_t workspace_bytes, uintptr_t stream,
           int row_group, int eos_token, float eos_threshold, uintptr_t probs_out,
           uintptr_t scores_out) {
          // AttentionCUDA::forward (attention/attention_cuda.cu:41-95) over a KVTileCache;
          // the filters and weight / score outputs of CPUAttentionInput / Output
          // (attention_cpu/attention_cpu.hpp:8-43) go through pa_decode_ex.
          pa_kv_view v;
          check(kv_cache_view(reinterpret_cast<kv_cache*>(kv_handle), layer, &v));
          const auto* qp = reinterpret_cast<const float*>(q);
          auto* op = reinterpret_cast<float*>(out);
          const auto* bi = reinterpret_cast<const int32_t*>(beam_ids);
          const auto* cl = reinterpret_cast<const int32_t*>(context_lens);
          void* ws = reinterpret_cast<void*>(workspace);
          void* st = reinterpret_cast<void*>(stream);
          if (top_k > 0 || top_p < 1.0f || eos_token >= 0 || probs_out || scores_out) {
            pa_decode_options o{temperature, top_k, top_p, eos_token, eos_threshold,
                                reinterpret_cast<float*>(probs_out),
                                reinterpret_cast<float*>(scores_out)};
            py::gil_scoped_release nogil;
            check(pa_decode_ex(&v, qp, op, bi, cl, B, H, D, T, &o, ws, workspace_bytes, st));
            return;
          }
          const float sm = 1.0f / (temperature * temperature);
          py::gil_scoped_release nogil;
          check(pa_decode_grouped(&v, qp, op, bi, cl, B, H, D, T, sm, 0, row_group, ws,
                                  workspace_bytes, st));
        },
        py::arg("kv_handle"), py::arg("layer"), py::arg("q"), py::arg("out"),
        py::arg("beam_ids") = 0, py::arg("context_lens") = 0, py::arg("B") = 1,
        py::arg("H") = 1, py::arg("D") = 64, py::arg("T") = 1, py::arg("temperature") = 1.0f,
        py::arg("top_k") = 0, py::arg("top_p") = 1.0f, py::arg("workspace") = 0,
        py::arg("workspace_bytes") = 0, py::arg("stream") = 0, py::arg("row_group") = 1,
        py::arg("eos_token") = -1, py::arg("eos_threshold") = 0.0f, py::arg("probs_out") = 0,
        py::arg("scores_out") = 0);
  m.def("dnnl_matmul_int8",
        [](uintptr_t A, uintptr_t B, uintptr_t C, int BATCH, int M, int N, int K, float scaleA,
           float scaleB, float scaleC, uintptr_t bias, const std::string& activation,
           uintptr_t stream) {
          // dnnl_matmul_int8 (attention_cpu/dnnl_matmul_int8.hpp:5-13): device
          // pointers; false on any failure, as the reference's catch (...) (:73-74);
          // an unknown activation adds no post-op (:44-50)
          const int act = activation == "relu" ? LLM_ACT_RELU
                          : activation == "gelu" ? LLM_ACT_GELU : LLM_ACT_NONE;
          py::gil_scoped_release nogil;
          return i8_matmul_s8(reinterpret_cast<const int8_t*>(A), reinterpret_cast<const int8_t*>(B),
                              reinterpret_cast<int8_t*>(C), BATCH, M, N, K, scaleA, scaleB, scaleC,
                              reinterpret_cast<const float*>(bias), act,
                              reinterpret_cast<void*>(stream)) == LLM_OK;
        },
        py::arg("A"), py::arg("B"), py::arg("C"), py::arg("BATCH"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("scaleA"), py::arg("scaleB"), py::arg("scaleC") = 1.0f,
        py::arg("bias") = 0, py::arg("activation") = "", py::arg("stream") = 0);
  m.def("workspace_bytes", &pa_decode_workspace_bytes, py::arg("B"), py::arg("H"), py::arg("D"),
        py::arg("max_tiles"), py::arg("pages_per_split") = 0);
  m.def("filter_workspace_bytes", &pa_decode_ex_workspace_bytes, py::arg("B"), py::arg("H"),
        py::arg("T"));
}
