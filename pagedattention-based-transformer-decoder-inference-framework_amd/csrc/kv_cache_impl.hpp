// Internal KV-cache state shared by kv_cache.cpp and the decoder runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <list>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "llm_decoder.h"

namespace llm {

struct KvCache {
  int L = 0, beams = 0, H = 0, D = 0, TS = 0, max_tiles = 0;
  long long num_pages = 0;
  int dtype = LLM_F16;  // pool element type
  int es = 2;           // bytes per element
  size_t page_elems = 0;
  size_t entries = 0;
  void* k_pool = nullptr;  // page p of K at k_pool + p * page_stride(), V right after it
  void* v_pool = nullptr;  // = k_pool + page_bytes() (same allocation)
  int32_t* d_table = nullptr;
  std::vector<int32_t> h_table;     // host mirror = source of truth
  std::vector<uint8_t> dirty_flag;
  std::vector<int64_t> dirty;
  std::vector<int32_t> refcount;
  // Free pages, one list per layer zone: page p belongs to zone
  // min(p / zone_pages, L - 1).  A layer allocates from its own zone first, so
  // the pages one attention launch gathers stay inside ~1/L of the pool (TLB
  // reach: a step walks every layer's pages once) — it falls back to the other
  // zones only when its own is exhausted.
  std::vector<std::vector<int32_t>> free_lists;
  long long zone_pages = 0;
  std::vector<std::pair<int32_t, int32_t>> cow;  // (src page, dst page) copies pending
  int64_t* d_idx = nullptr;
  int32_t* d_val = nullptr;
  int64_t* h_idx = nullptr;
  int32_t* h_val = nullptr;
  size_t staging_cap = 0;
  hipEvent_t staging_done = nullptr;
  std::mutex mu;
  // kv_cache_set_eviction: LLM_EVICT_LRU makes register_tile evict the least
  // recently registered table entries when the pool is exhausted
  // (kv_tile_cache.cpp:79-98).  lru: the table indices register_tile mapped,
  // most recent first.  Any other write of an entry (set_entry: reserve /
  // prepare_append, assign, remove, release, fork, COW, snapshot load) drops
  // it from the list, so a page a later caller puts on that entry is never an
  // eviction candidate unless register_tile maps it again.
  int evict = LLM_EVICT_NONE;
  std::list<size_t> lru;
  std::unordered_map<size_t, std::list<size_t>::iterator> lru_pos;
  void lru_touch(size_t idx);
  void lru_forget(size_t idx);
  bool lru_evict_one();  // false: nothing left to evict

  ~KvCache();
  int init(int L, int beams, int H, int D, int TS, int max_tiles, long long pages,
           int dtype = LLM_F16);
  size_t page_bytes() const { return page_elems * es; }
  size_t page_stride() const { return 2 * page_bytes(); }  // K and V pages interleave
  size_t index(int layer, int beam, int head, int tile) const {
    return (((size_t)layer * beams + beam) * H + head) * max_tiles + tile;
  }
  bool in_range(int layer, int beam, int head, int tile) const;
  void set_entry(size_t idx, int32_t page);
  int zone_of_page(int32_t page) const {
    return (int)std::min<long long>(page / zone_pages, (long long)free_lists.size() - 1);
  }
  int zone_of_layer(int layer) const { return std::min(layer, (int)free_lists.size() - 1); }
  void reset_free_lists();
  long long free_count() const;
  bool take_free(int32_t page);  // remove a specific page from its free list
  int alloc_page(int layer, int32_t* out);
  void drop_page(int32_t page);
  // allocate (and, if exclusive, un-share by copy-on-write) the page of a tile
  int ensure_tile(int layer, int beam, int head, int tile, bool exclusive, int32_t* page);
  // make the tile of `pos` exist and be exclusive for every layer / head of `beam`
  int prepare_append(int beam, int pos);
  // push copy-on-write copies and dirty table entries to the device (stream-ordered)
  int sync(hipStream_t st);
};

}  // namespace llm

struct kv_cache {
  llm::KvCache impl;
};
llm::KvCache* kv_impl(kv_cache* c);
