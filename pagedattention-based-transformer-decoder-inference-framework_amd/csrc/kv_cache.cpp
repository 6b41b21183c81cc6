// KV page pools + page table (host runtime), compiled as HIP.
//
// Replaces PageTable (kv_cache/page_table.{hpp,cpp}) and KVTileCache<T>
// (kv_cache/kv_tile_cache.{hpp,cpp}) with:
//   * a layer dimension: table [L][beams][H][max_tiles] (the reference shares
//     one table across layers, Appendix A #11, and sizes it (pages, D, ts),
//     kv_tile_cache.cpp:23 — both defects);
//   * ONE source of truth: the host mirror; the device table is updated by
//     kv_cache_sync() with a scatter of the dirty entries (the reference's
//     assign() writes only the device, remove() only the host, and
//     sync_to_gpu() overwrites the device, page_table.cpp:49-66);
//   * a free-list page allocator (one list per layer zone) with per-page refcounts (the reference's
//     page id = map.size() aliases live pages after an eviction,
//     kv_tile_cache.cpp:71), so beams can fork and share prefix pages;
//   * copy-on-write of a shared page before a token is written into it.
// The K and V pools interleave page by page in ONE hipMalloc:
// [num_pages][K page | V page], so page p's K and V are adjacent (see
// KvCache::init), sized for the 288 GB HBM of an MI355X (page ids are int32,
// byte offsets 64-bit).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "kv_cache_impl.hpp"
#include "row_ops.hpp"

namespace llm {

// src [n][H][D] rows (element type E) for token positions pos0..pos0+n-1 of `beam`.
template <typename E>
__global__ void kv_write_tokens_kernel(const E* __restrict__ ksrc, const E* __restrict__ vsrc,
                                       int n, int H, int D, int pos0, int beam,
                                       const int32_t* __restrict__ table, int max_tiles, int TS,
                                       long long num_pages, size_t page_stride, E* __restrict__ kp,
                                       E* __restrict__ vp) {
  const size_t total = (size_t)n * H * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int d = i % D;
    const int h = (i / D) % H;
    const int t = i / ((size_t)H * D);
    const int pos = pos0 + t;
    const int tile = pos / TS;
    if (tile >= max_tiles) continue;
    const int page = table[((size_t)beam * H + h) * max_tiles + tile];
    if (page < 0 || page >= num_pages) continue;
    const size_t off = (size_t)page * page_stride + (size_t)(pos % TS) * D + d;
    kp[off] = ksrc[i];
    vp[off] = vsrc[i];
  }
}

int KvCache::init(int L_, int beams_, int H_, int D_, int TS_, int max_tiles_, long long pages,
                  int dtype_) {
  L = L_; beams = beams_; H = H_; D = D_; TS = TS_; max_tiles = max_tiles_; num_pages = pages;
  dtype = dtype_;
  es = dtype == LLM_F32 ? 4 : dtype == LLM_I8 ? 1 : 2;
  page_elems = (size_t)TS * D;
  // A wave loads K page p and V page p together.  With two separate pools at
  // a large distance the pair often falls into the same HBM channel and the
  // scan loses 2-4 %, depending on the distance (C3 shape,
  // scripts/tune_attention.py --v-gap: 648-685 us across V-pool offsets);
  // adjacent K / V pages measured 649 us at every context length tried
  // (--interleave).
  const size_t alloc = (size_t)num_pages * page_stride();
  if (hipMalloc(&k_pool, alloc) != hipSuccess) {
    (void)hipGetLastError();
    return fail(LLM_ERR_OOM, "kv_cache: cannot allocate " + std::to_string(alloc) +
                                 " bytes of page pool");
  }
  v_pool = static_cast<char*>(k_pool) + page_bytes();
  entries = (size_t)L * beams * H * max_tiles;
  LLM_HIP_RET(hipMalloc(&d_table, entries * sizeof(int32_t)));
  LLM_HIP_RET(hipMemset(d_table, 0xFF, entries * sizeof(int32_t)));  // -1 (page_table.cpp:22-25)
  LLM_HIP_RET(hipDeviceSynchronize());  // null-stream memset vs. non-blocking user streams
  h_table.assign(entries, -1);
  dirty_flag.assign(entries, 0);
  refcount.assign((size_t)num_pages, 0);
  reset_free_lists();
  LLM_HIP_RET(hipEventCreateWithFlags(&staging_done, hipEventDisableTiming));
  return LLM_OK;
}

KvCache::~KvCache() {
  if (staging_done) (void)hipEventSynchronize(staging_done);
  if (k_pool) (void)hipFree(k_pool);  // v_pool lives in the same allocation
  if (d_table) (void)hipFree(d_table);
  if (d_idx) (void)hipFree(d_idx);
  if (d_val) (void)hipFree(d_val);
  if (h_idx) (void)hipHostFree(h_idx);
  if (h_val) (void)hipHostFree(h_val);
  if (staging_done) (void)hipEventDestroy(staging_done);
}

bool KvCache::in_range(int layer, int beam, int head, int tile) const {
  return layer >= 0 && layer < L && beam >= 0 && beam < beams && head >= 0 && head < H &&
         tile >= 0 && tile < max_tiles;
}

void KvCache::set_entry(size_t idx, int32_t page) {
  h_table[idx] = page;
  lru_forget(idx);  // register_tile re-adds the entries it maps (lru_touch after this)
  if (!dirty_flag[idx]) {
    dirty_flag[idx] = 1;
    dirty.push_back((int64_t)idx);
  }
}

void KvCache::reset_free_lists() {
  const int zones = (int)std::max<long long>(1, std::min<long long>(L, num_pages));
  zone_pages = num_pages / zones;
  free_lists.assign(zones, {});
  for (long long p = num_pages - 1; p >= 0; --p)  // pop_back hands out low ids first
    if (refcount[p] == 0) free_lists[zone_of_page((int32_t)p)].push_back((int32_t)p);
}

long long KvCache::free_count() const {
  long long n = 0;
  for (const auto& f : free_lists) n += (long long)f.size();
  return n;
}

bool KvCache::take_free(int32_t page) {
  auto& f = free_lists[zone_of_page(page)];
  auto it = std::find(f.begin(), f.end(), page);
  if (it == f.end()) return false;
  f.erase(it);
  return true;
}

int KvCache::alloc_page(int layer, int32_t* out) {
  const int z0 = zone_of_layer(std::max(layer, 0));
  const int nz = (int)free_lists.size();
  for (int i = 0; i < nz; ++i) {
    auto& f = free_lists[(z0 + i) % nz];
    if (f.empty()) continue;
    *out = f.back();
    f.pop_back();
    refcount[*out] = 1;
    return LLM_OK;
  }
  return fail(LLM_ERR_OOM, "kv_cache: page pool exhausted (" + std::to_string(num_pages) +
                               " pages)");
}

void KvCache::drop_page(int32_t page) {
  if (page < 0 || page >= num_pages) return;
  if (--refcount[page] <= 0) {
    refcount[page] = 0;
    free_lists[zone_of_page(page)].push_back(page);
  }
}

int KvCache::ensure_tile(int layer, int beam, int head, int tile, bool exclusive, int32_t* page) {
  const size_t idx = index(layer, beam, head, tile);
  int32_t p = h_table[idx];
  if (p < 0) {
    int rc = alloc_page(layer, &p);
    if (rc) return rc;
    set_entry(idx, p);
  } else if (exclusive && refcount[p] > 1) {
    // copy-on-write: the page is shared with a forked beam
    int32_t np;
    int rc = alloc_page(layer, &np);
    if (rc) return rc;
    cow.push_back({p, np});
    refcount[p] -= 1;
    set_entry(idx, np);
    p = np;
  }
  if (page) *page = p;
  return LLM_OK;
}

void KvCache::lru_touch(size_t idx) {  // KVTileCache::update_lru, kv_tile_cache.cpp:79-87
  auto it = lru_pos.find(idx);
  if (it != lru_pos.end()) lru.erase(it->second);
  lru.push_front(idx);
  lru_pos[idx] = lru.begin();
}

void KvCache::lru_forget(size_t idx) {
  if (lru_pos.empty()) return;
  auto it = lru_pos.find(idx);
  if (it == lru_pos.end()) return;
  lru.erase(it->second);
  lru_pos.erase(it);
}

// KVTileCache::evict_if_needed (kv_tile_cache.cpp:89-98): remove the least
// recently registered entry whose page that frees.  Only entries register_tile
// mapped are in the list (set_entry drops any entry another call rewrites);
// entries on a page a forked beam
// still shares stay (evicting them would free nothing, and the reference has
// no shared pages), so a pool held only by shared pages still reports OOM.
bool KvCache::lru_evict_one() {
  for (auto it = lru.end(); it != lru.begin();) {
    --it;
    const size_t idx = *it;
    const int32_t p = h_table[idx];
    if (p >= 0 && refcount[p] > 1) continue;
    lru_pos.erase(idx);
    it = lru.erase(it);
    if (p < 0) continue;  // (not reached: set_entry drops unmapped entries)
    drop_page(p);
    set_entry(idx, -1);
    return true;
  }
  return false;
}

int KvCache::prepare_append(int beam, int pos) {
  const int tile = pos / TS;
  if (tile >= max_tiles)
    return fail(LLM_ERR_INVALID, "kv_cache: position " + std::to_string(pos) +
                                     " beyond max_tiles*page_size");
  for (int l = 0; l < L; ++l)
    for (int h = 0; h < H; ++h) {
      int rc = ensure_tile(l, beam, h, tile, true, nullptr);
      if (rc) return rc;
    }
  return LLM_OK;
}

int KvCache::sync(hipStream_t st) {
  // pending copy-on-write page copies first (old page -> new page; K and V
  // are adjacent, one copy each)
  for (const auto& c : cow) {
    const size_t bytes = page_stride();
    LLM_HIP_RET(hipMemcpyAsync((char*)k_pool + (size_t)c.second * bytes,
                               (char*)k_pool + (size_t)c.first * bytes, bytes,
                               hipMemcpyDeviceToDevice, st));
  }
  cow.clear();
  if (dirty.empty()) return LLM_OK;
  const size_t n = dirty.size();
  if (n * 4 > entries) {  // mostly dirty: push the whole table
    LLM_HIP_RET(hipEventSynchronize(staging_done));
    LLM_HIP_RET(hipMemcpyAsync(d_table, h_table.data(), entries * sizeof(int32_t),
                               hipMemcpyHostToDevice, st));
    LLM_HIP_RET(hipStreamSynchronize(st));  // pageable source: keep it valid until copied
  } else {
    LLM_HIP_RET(hipEventSynchronize(staging_done));  // previous staging consumed
    if (n > staging_cap) {
      if (d_idx) LLM_HIP_RET(hipFree(d_idx));
      if (d_val) LLM_HIP_RET(hipFree(d_val));
      if (h_idx) LLM_HIP_RET(hipHostFree(h_idx));
      if (h_val) LLM_HIP_RET(hipHostFree(h_val));
      staging_cap = std::max<size_t>(n, 4096);
      LLM_HIP_RET(hipMalloc(&d_idx, staging_cap * sizeof(int64_t)));
      LLM_HIP_RET(hipMalloc(&d_val, staging_cap * sizeof(int32_t)));
      LLM_HIP_RET(hipHostMalloc(&h_idx, staging_cap * sizeof(int64_t), hipHostMallocDefault));
      LLM_HIP_RET(hipHostMalloc(&h_val, staging_cap * sizeof(int32_t), hipHostMallocDefault));
    }
    for (size_t i = 0; i < n; ++i) {
      h_idx[i] = dirty[i];
      h_val[i] = h_table[dirty[i]];
    }
    LLM_HIP_RET(hipMemcpyAsync(d_idx, h_idx, n * sizeof(int64_t), hipMemcpyHostToDevice, st));
    LLM_HIP_RET(hipMemcpyAsync(d_val, h_val, n * sizeof(int32_t), hipMemcpyHostToDevice, st));
    LLM_HIP_RET(launch_scatter_i32(d_table, d_idx, d_val, (int)n, st));
    LLM_HIP_RET(hipEventRecord(staging_done, st));
  }
  for (int64_t i : dirty) dirty_flag[i] = 0;
  dirty.clear();
  return LLM_OK;
}

}  // namespace llm

using namespace llm;

extern "C" int kv_cache_create(int num_layers, int num_beams, int num_heads, int head_dim,
                               int page_size, int max_tiles, long long num_pages, kv_cache** out) {
  return kv_cache_create_typed(num_layers, num_beams, num_heads, head_dim, page_size, max_tiles,
                               num_pages, LLM_F16, out);
}

extern "C" int kv_cache_create_typed(int num_layers, int num_beams, int num_heads, int head_dim,
                                     int page_size, int max_tiles, long long num_pages,
                                     int kv_dtype, kv_cache** out) {
  LLM_REQUIRE(out != nullptr, "kv_cache_create: out is NULL");
  LLM_REQUIRE(kv_dtype == LLM_F16 || kv_dtype == LLM_BF16 || kv_dtype == LLM_F32 ||
                  kv_dtype == LLM_I8,
              "kv_cache_create: kv_dtype must be LLM_F16, LLM_BF16, LLM_F32 or LLM_I8");
  LLM_REQUIRE(num_layers > 0 && num_beams > 0 && num_heads > 0 && head_dim > 0 && page_size > 0 &&
                  max_tiles > 0 && num_pages > 0,
              "kv_cache_create: all sizes must be positive");
  LLM_REQUIRE(num_pages < (1LL << 31), "kv_cache_create: num_pages must fit int32");
  auto* c = new kv_cache();
  int rc = c->impl.init(num_layers, num_beams, num_heads, head_dim, page_size, max_tiles, num_pages,
                        kv_dtype);
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return LLM_OK;
}

extern "C" void kv_cache_destroy(kv_cache* c) { delete c; }

KvCache* kv_impl(kv_cache* c) { return c ? &c->impl : nullptr; }

extern "C" int kv_cache_view(const kv_cache* c, int layer, pa_kv_view* out) {
  LLM_REQUIRE(c && out, "kv_cache_view: NULL");
  const KvCache& k = c->impl;
  LLM_REQUIRE(layer >= 0 && layer < k.L, "kv_cache_view: bad layer");
  out->k_pool = k.k_pool;
  out->v_pool = k.v_pool;
  out->page_table = k.d_table + (size_t)layer * k.beams * k.H * k.max_tiles;
  out->num_pages = (int32_t)k.num_pages;
  out->page_size = k.TS;
  out->head_dim = k.D;
  out->num_beams = k.beams;
  out->page_stride = (int64_t)k.page_stride();
  out->num_heads = k.H;
  out->max_tiles = k.max_tiles;
  out->kv_dtype = k.dtype;
  return LLM_OK;
}

extern "C" long long kv_cache_num_pages(const kv_cache* c) { return c ? c->impl.num_pages : -1; }

extern "C" long long kv_cache_free_pages(const kv_cache* c) {
  if (!c) return -1;
  std::lock_guard<std::mutex> g(const_cast<kv_cache*>(c)->impl.mu);
  return c->impl.free_count();
}

extern "C" int kv_cache_assign(kv_cache* c, int layer, int beam, int head, int tile, int page) {
  LLM_REQUIRE(c, "kv_cache_assign: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(k.in_range(layer, beam, head, tile), "kv_cache_assign: index out of range");
  LLM_REQUIRE(page >= -1 && page < k.num_pages, "kv_cache_assign: page out of range");
  const size_t idx = k.index(layer, beam, head, tile);
  const int32_t old = k.h_table[idx];
  k.lru_forget(idx);  // an entry set by hand is not a registered tile (no eviction candidate)
  if (old == page) return LLM_OK;
  if (page >= 0) {
    // take the page out of the free list if it is there; bump its refcount
    k.take_free(page);
    k.refcount[page] += 1;
  }
  k.drop_page(old);
  k.set_entry(idx, page);
  return LLM_OK;
}

extern "C" int kv_cache_lookup(const kv_cache* c, int layer, int beam, int head, int tile) {
  if (!c) return -1;
  const KvCache& k = c->impl;
  if (!k.in_range(layer, beam, head, tile)) return -1;  // page_table.hpp:47
  return k.h_table[k.index(layer, beam, head, tile)];
}

extern "C" int kv_cache_remove(kv_cache* c, int layer, int beam, int head, int tile) {
  return kv_cache_assign(c, layer, beam, head, tile, -1);
}

extern "C" int kv_cache_register_tile(kv_cache* c, int layer, int beam, int head, int tile,
                                      int* page) {
  LLM_REQUIRE(c, "kv_cache_register_tile: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(k.in_range(layer, beam, head, tile), "kv_cache_register_tile: index out of range");
  const size_t idx = k.index(layer, beam, head, tile);
  int32_t p;
  int rc = k.ensure_tile(layer, beam, head, tile, false, &p);
  // LRU policy: a tile without a page takes one by evicting the least recently
  // registered entries (an entry sharing a forked page frees nothing, so the
  // next one goes too) until a page is free or nothing is left to evict
  while (rc == LLM_ERR_OOM && k.evict == LLM_EVICT_LRU && k.lru_evict_one())
    rc = k.ensure_tile(layer, beam, head, tile, false, &p);
  if (rc) return rc;
  k.lru_touch(idx);  // (under either policy, so switching to LRU later sees the order)
  if (page) *page = p;
  return LLM_OK;
}

extern "C" int kv_cache_set_eviction(kv_cache* c, int policy) {
  LLM_REQUIRE(c, "kv_cache_set_eviction: NULL");
  LLM_REQUIRE(policy == LLM_EVICT_NONE || policy == LLM_EVICT_LRU,
              "kv_cache_set_eviction: policy must be LLM_EVICT_NONE or LLM_EVICT_LRU");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  k.evict = policy;
  return LLM_OK;
}

extern "C" int kv_cache_reserve(kv_cache* c, int beam, int n_tokens) {
  LLM_REQUIRE(c, "kv_cache_reserve: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(beam >= 0 && beam < k.beams && n_tokens >= 0, "kv_cache_reserve: bad beam/n");
  const int nt = (n_tokens + k.TS - 1) / k.TS;
  LLM_REQUIRE(nt <= k.max_tiles, "kv_cache_reserve: n_tokens exceeds max_tiles*page_size");
  for (int l = 0; l < k.L; ++l)
    for (int h = 0; h < k.H; ++h)
      for (int t = 0; t < nt; ++t) {
        int rc = k.ensure_tile(l, beam, h, t, false, nullptr);
        if (rc) return rc;
      }
  return LLM_OK;
}

extern "C" int kv_cache_fork(kv_cache* c, int src_beam, int dst_beam) {
  LLM_REQUIRE(c, "kv_cache_fork: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(src_beam >= 0 && src_beam < k.beams && dst_beam >= 0 && dst_beam < k.beams,
              "kv_cache_fork: bad beam");
  if (src_beam == dst_beam) return LLM_OK;
  for (int l = 0; l < k.L; ++l)
    for (int h = 0; h < k.H; ++h)
      for (int t = 0; t < k.max_tiles; ++t) {
        const size_t si = k.index(l, src_beam, h, t), di = k.index(l, dst_beam, h, t);
        const int32_t sp = k.h_table[si], dp = k.h_table[di];
        if (sp == dp) continue;
        if (sp >= 0) k.refcount[sp] += 1;
        k.drop_page(dp);
        k.set_entry(di, sp);
      }
  return LLM_OK;
}

extern "C" int kv_cache_release(kv_cache* c, int beam) {
  LLM_REQUIRE(c, "kv_cache_release: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(beam >= 0 && beam < k.beams, "kv_cache_release: bad beam");
  for (int l = 0; l < k.L; ++l)
    for (int h = 0; h < k.H; ++h)
      for (int t = 0; t < k.max_tiles; ++t) {
        const size_t i = k.index(l, beam, h, t);
        if (k.h_table[i] >= 0) {
          k.drop_page(k.h_table[i]);
          k.set_entry(i, -1);
        }
      }
  return LLM_OK;
}

extern "C" int kv_cache_clear(kv_cache* c) {
  LLM_REQUIRE(c, "kv_cache_clear: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_HIP_RET(hipEventSynchronize(k.staging_done));
  std::fill(k.h_table.begin(), k.h_table.end(), -1);
  std::fill(k.dirty_flag.begin(), k.dirty_flag.end(), 0);
  k.dirty.clear();
  k.cow.clear();
  std::fill(k.refcount.begin(), k.refcount.end(), 0);
  k.reset_free_lists();
  k.lru.clear();
  k.lru_pos.clear();
  LLM_HIP_RET(hipMemset(k.d_table, 0xFF, k.entries * sizeof(int32_t)));
  LLM_HIP_RET(hipDeviceSynchronize());  // null-stream memset vs. non-blocking user streams
  return LLM_OK;
}

extern "C" int kv_cache_sync(kv_cache* c, void* stream) {
  LLM_REQUIRE(c, "kv_cache_sync: NULL");
  std::lock_guard<std::mutex> g(c->impl.mu);
  return c->impl.sync(as_stream(stream));
}

extern "C" int kv_cache_write_tokens(kv_cache* c, int layer, int beam, int pos, int n,
                                     const void* k_host, const void* v_host) {
  LLM_REQUIRE(c && k_host && v_host, "kv_cache_write_tokens: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  LLM_REQUIRE(layer >= 0 && layer < k.L && beam >= 0 && beam < k.beams && pos >= 0 && n >= 0,
              "kv_cache_write_tokens: bad arguments");
  if (n == 0) return LLM_OK;
  LLM_REQUIRE((pos + n + k.TS - 1) / k.TS <= k.max_tiles,
              "kv_cache_write_tokens: tokens beyond max_tiles*page_size");
  // every target tile must exist and be exclusively owned (copy-on-write)
  for (int t = pos / k.TS; t <= (pos + n - 1) / k.TS; ++t)
    for (int h = 0; h < k.H; ++h) {
      int rc = k.ensure_tile(layer, beam, h, t, true, nullptr);
      if (rc) return rc;
    }
  int rc = k.sync(nullptr);
  if (rc) return rc;
  const size_t bytes = (size_t)n * k.H * k.D * k.es;
  void *dk = nullptr, *dv = nullptr;
  LLM_HIP_RET(hipMalloc(&dk, bytes));
  LLM_HIP_RET(hipMalloc(&dv, bytes));
  LLM_HIP_RET(hipMemcpy(dk, k_host, bytes, hipMemcpyHostToDevice));
  LLM_HIP_RET(hipMemcpy(dv, v_host, bytes, hipMemcpyHostToDevice));
  const size_t total = (size_t)n * k.H * k.D;
  const dim3 grid((unsigned)std::min<size_t>((total + 255) / 256, 65536));
  const int32_t* table = k.d_table + (size_t)layer * k.beams * k.H * k.max_tiles;
  auto launch = [&](auto tag) {
    using E = decltype(tag);
    hipLaunchKernelGGL(kv_write_tokens_kernel<E>, grid, dim3(256), 0, nullptr,
                       static_cast<const E*>(dk), static_cast<const E*>(dv), n, k.H, k.D, pos,
                       beam, table, k.max_tiles, k.TS, k.num_pages, k.page_stride() / k.es,
                       static_cast<E*>(k.k_pool), static_cast<E*>(k.v_pool));
  };
  if (k.es == 4) launch(uint32_t{});
  else if (k.es == 1) launch(uint8_t{});
  else launch(uint16_t{});
  LLM_HIP_RET(hipGetLastError());
  LLM_HIP_RET(hipDeviceSynchronize());
  LLM_HIP_RET(hipFree(dk));
  LLM_HIP_RET(hipFree(dv));
  return LLM_OK;
}

extern "C" void* kv_cache_k_pool(kv_cache* c) { return c ? c->impl.k_pool : nullptr; }
extern "C" void* kv_cache_v_pool(kv_cache* c) { return c ? c->impl.v_pool : nullptr; }
extern "C" long long kv_cache_page_stride(const kv_cache* c) {
  return c ? (long long)c->impl.page_stride() : 0;
}
extern "C" int32_t* kv_cache_page_table(kv_cache* c, int layer) {
  if (!c || layer < 0 || layer >= c->impl.L) return nullptr;
  const KvCache& k = c->impl;
  return k.d_table + (size_t)layer * k.beams * k.H * k.max_tiles;
}
