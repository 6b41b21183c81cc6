// KV cache files (host runtime + two copy kernels), compiled as HIP.
//
// Three on-disk formats:
//   * the reference's pool dump, KVTileCache<T>::save_to_file / load_from_file
//     (kv_cache/kv_tile_cache.cpp:105-125): the raw K pool [pages][ts][D] then
//     the raw V pool, nothing else (the page table is not saved; the reader
//     keeps its own) -> kv_cache_save_pools / kv_cache_load_pools;
//   * the reference's tile records, KVTileCacheCPU<T>::save / load
//     (kv_cache/kv_tile_cache_cpu.cpp:89-123): int32 count, then per tile
//     {int32 batch_id, head_id, tile_id} + tile_size_ elements of T.  K and V
//     live in two such caches, so one file holds one of them
//     for one layer -> kv_cache_save_tiles / kv_cache_load_tiles;
//   * this build's snapshot "APPIMKV2": geometry header, the whole layered page
//     table and every used page (K then V) -> kv_cache_save / kv_cache_load.
// Every reader validates the whole file (sizes, ids, table entries) before it
// changes the cache; kv_tiles_inspect / kv_cache_inspect run that validation
// alone, on the host, without a device.
#include <algorithm>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "kv_cache_impl.hpp"

using namespace llm;

namespace {

constexpr uint64_t kMagic = 0x31564B4D49505041ull;    // "APPIMKV1": fp16 pools, 8-word header
constexpr uint64_t kMagicV2 = 0x32564B4D49505041ull;  // "APPIMKV2": + kv_dtype word
constexpr size_t kStagingBytes = 64ull << 20;         // host/device staging per chunk

int elem_bytes(int dtype) { return dtype == LLM_F32 ? 4 : dtype == LLM_I8 ? 1 : 2; }

long long file_size(std::ifstream& f) {
  f.seekg(0, std::ios::end);
  const long long n = (long long)f.tellg();
  f.seekg(0, std::ios::beg);
  return n;
}

// Copy n blocks of `bytes` between a dense staging buffer and pool pages:
// block i <-> base + ids[i] * stride (ids[i] < 0: skipped).  V = 16-byte
// vectors when every size and offset allows, else bytes.
template <typename V, bool kToPool>
__global__ void page_copy_kernel(V* __restrict__ dense, char* __restrict__ base,
                                 const int64_t* __restrict__ ids, int n, size_t bytes,
                                 size_t stride) {
  const size_t per = bytes / sizeof(V);
  const size_t total = (size_t)n * per;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t blk = i / per, e = i % per;
    const int64_t id = ids[blk];
    if (id < 0) continue;
    V* pool = reinterpret_cast<V*>(base + (size_t)id * stride) + e;
    if constexpr (kToPool) *pool = dense[i];
    else dense[i] = *pool;
  }
}

// Staging for chunked page copies (one device buffer + id list, reused).
struct PageMover {
  void* d_dense = nullptr;
  int64_t* d_ids = nullptr;
  size_t cap_bytes = 0;
  int cap_ids = 0;
  ~PageMover() {
    if (d_dense) (void)hipFree(d_dense);
    if (d_ids) (void)hipFree(d_ids);
  }
  int reserve(size_t bytes, int ids) {
    if (bytes > cap_bytes) {
      if (d_dense) LLM_HIP_RET(hipFree(d_dense));
      d_dense = nullptr;
      LLM_HIP_RET(hipMalloc(&d_dense, bytes));
      cap_bytes = bytes;
    }
    if (ids > cap_ids) {
      if (d_ids) LLM_HIP_RET(hipFree(d_ids));
      d_ids = nullptr;
      LLM_HIP_RET(hipMalloc(&d_ids, (size_t)ids * sizeof(int64_t)));
      cap_ids = ids;
    }
    return LLM_OK;
  }
  // host dense <-> pool blocks base + ids[i] * stride, `bytes` each
  int move(bool to_pool, void* host_dense, char* base, const std::vector<int64_t>& ids,
           size_t bytes, size_t stride) {
    const int n = (int)ids.size();
    if (n == 0) return LLM_OK;
    if (int rc = reserve(bytes * n, n)) return rc;
    LLM_HIP_RET(hipMemcpy(d_ids, ids.data(), n * sizeof(int64_t), hipMemcpyHostToDevice));
    if (to_pool)
      LLM_HIP_RET(hipMemcpy(d_dense, host_dense, bytes * n, hipMemcpyHostToDevice));
    const bool vec = bytes % 16 == 0 && stride % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(base) % 16 == 0;
    const size_t per = vec ? bytes / 16 : bytes;
    const dim3 grid((unsigned)std::min<size_t>((per * n + 255) / 256, 16384)), blk(256);
    if (vec) {
      if (to_pool)
        hipLaunchKernelGGL((page_copy_kernel<uint4, true>), grid, blk, 0, nullptr,
                           static_cast<uint4*>(d_dense), base, d_ids, n, bytes, stride);
      else
        hipLaunchKernelGGL((page_copy_kernel<uint4, false>), grid, blk, 0, nullptr,
                           static_cast<uint4*>(d_dense), base, d_ids, n, bytes, stride);
    } else {
      if (to_pool)
        hipLaunchKernelGGL((page_copy_kernel<uint8_t, true>), grid, blk, 0, nullptr,
                           static_cast<uint8_t*>(d_dense), base, d_ids, n, bytes, stride);
      else
        hipLaunchKernelGGL((page_copy_kernel<uint8_t, false>), grid, blk, 0, nullptr,
                           static_cast<uint8_t*>(d_dense), base, d_ids, n, bytes, stride);
    }
    LLM_HIP_RET(hipGetLastError());
    if (!to_pool)
      LLM_HIP_RET(hipMemcpy(host_dense, d_dense, bytes * n, hipMemcpyDeviceToHost));
    LLM_HIP_RET(hipDeviceSynchronize());
    return LLM_OK;
  }
};

// ---------------------------------------------------------------------------
// snapshot (APPIMKV2) parsing: everything but the page bytes, fully checked
// ---------------------------------------------------------------------------
struct Snapshot {
  int64_t geo[8] = {};  // L, beams, H, D, TS, max_tiles, num_pages, dtype
  std::vector<int32_t> table;
  std::vector<int32_t> used;
  long long data_off = 0;
  size_t page_bytes = 0;
};

int parse_snapshot(std::ifstream& f, const char* path, Snapshot& s) {
  const std::string p = path;
  const long long size = file_size(f);
  int64_t hdr[8];
  f.read(reinterpret_cast<char*>(hdr), sizeof(hdr));
  if (!f || (hdr[0] != (int64_t)kMagic && hdr[0] != (int64_t)kMagicV2))
    return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": bad header");
  long long off = (long long)sizeof(hdr);
  for (int i = 0; i < 7; ++i) s.geo[i] = hdr[i + 1];
  s.geo[7] = LLM_F16;
  if (hdr[0] == (int64_t)kMagicV2) {
    f.read(reinterpret_cast<char*>(&s.geo[7]), sizeof(int64_t));
    off += sizeof(int64_t);
    if (!f) return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": bad header");
  }
  const int64_t L = s.geo[0], beams = s.geo[1], H = s.geo[2], D = s.geo[3], TS = s.geo[4],
                mt = s.geo[5], np = s.geo[6], dt = s.geo[7];
  if (L <= 0 || beams <= 0 || H <= 0 || D <= 0 || TS <= 0 || mt <= 0 || np <= 0 ||
      np >= (1LL << 31) || D > (1 << 16) || TS > (1 << 16) || TS * D > (1 << 24) || (dt != LLM_F16 && dt != LLM_BF16 && dt != LLM_F32 && dt != LLM_I8))
    return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": bad geometry");
  // entries * 4 must fit in the file before anything is allocated
  const long long room = (size - off) / 4;
  if (L > room || beams > room / L || H > room / (L * beams) || mt > room / (L * beams * H))
    return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": truncated page table");
  const size_t entries = (size_t)(L * beams * H * mt);
  s.page_bytes = (size_t)TS * D * elem_bytes((int)dt);
  s.table.resize(entries);
  f.read(reinterpret_cast<char*>(s.table.data()), entries * sizeof(int32_t));
  int64_t nu = -1;
  f.read(reinterpret_cast<char*>(&nu), sizeof(nu));
  if (!f) return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": truncated page table");
  off += (long long)entries * 4 + 8;
  if (nu < 0 || nu > np || nu > (size - off) / 4)
    return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": bad used-page count");
  s.used.resize((size_t)nu);
  f.read(reinterpret_cast<char*>(s.used.data()), (size_t)nu * sizeof(int32_t));
  if (!f) return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": truncated used-page list");
  off += nu * 4;
  for (int64_t i = 0; i < nu; ++i)
    if (s.used[i] < 0 || s.used[i] >= np || (i > 0 && s.used[i] <= s.used[i - 1]))
      return fail(LLM_ERR_IO, "kv_cache snapshot " + p +
                                  ": used-page ids must be ascending and inside the pool");
  for (int32_t t : s.table) {
    if (t < -1 || t >= np)
      return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": page-table entry outside the pool");
    if (t >= 0 && !std::binary_search(s.used.begin(), s.used.end(), t))
      return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": page-table entry names an unsaved page");
  }
  if ((unsigned long long)(size - off) != (unsigned long long)nu * 2 * s.page_bytes)
    return fail(LLM_ERR_IO, "kv_cache snapshot " + p + ": page data size does not match (" +
                                std::to_string(size - off) + " bytes for " + std::to_string(nu) +
                                " pages)");
  s.data_off = off;
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// tile-record file (KVTileCacheCPU::save) parsing: the index list, checked
// ---------------------------------------------------------------------------
int parse_tiles(std::ifstream& f, const char* path, long long tile_bytes,
                std::vector<int32_t>* idx, int* count) {
  const std::string p = path;
  const long long size = file_size(f);
  int32_t n = -1;
  f.read(reinterpret_cast<char*>(&n), sizeof(n));
  if (!f || n < 0) return fail(LLM_ERR_IO, "kv tile file " + p + ": bad record count");
  const long long rec = 12 + tile_bytes;
  if (size != 4 + (long long)n * rec)
    return fail(LLM_ERR_IO, "kv tile file " + p + ": " + std::to_string(size) +
                                " bytes, expected 4 + " + std::to_string(n) + " x " +
                                std::to_string(rec) + " (count x (12-byte index + tile))");
  if (idx) {
    idx->resize((size_t)n * 3);
    for (int32_t i = 0; i < n; ++i) {
      f.seekg(4 + (long long)i * rec);
      f.read(reinterpret_cast<char*>(idx->data() + 3 * (size_t)i), 12);
    }
    if (!f) return fail(LLM_ERR_IO, "kv tile file " + p + ": read failed");
  }
  *count = n;
  return LLM_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// host-only inspection (no device needed)
// ---------------------------------------------------------------------------
extern "C" int kv_tiles_inspect(const char* path, long long tile_bytes, int* count) {
  LLM_REQUIRE(path && count && tile_bytes > 0, "kv_tiles_inspect: bad arguments");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_tiles_inspect: cannot open ") + path);
  std::vector<int32_t> idx;
  int n = 0;
  if (int rc = parse_tiles(f, path, tile_bytes, &idx, &n)) return rc;
  for (int i = 0; i < 3 * n; ++i)
    if (idx[i] < 0) return fail(LLM_ERR_IO, std::string("kv_tiles_inspect: negative index in ") + path);
  *count = n;
  return LLM_OK;
}

extern "C" int kv_cache_inspect(const char* path, long long* geometry) {
  LLM_REQUIRE(path && geometry, "kv_cache_inspect: NULL");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_inspect: cannot open ") + path);
  Snapshot s;
  if (int rc = parse_snapshot(f, path, s)) return rc;
  for (int i = 0; i < 8; ++i) geometry[i] = s.geo[i];
  geometry[8] = (long long)s.used.size();
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// snapshot save / load
// ---------------------------------------------------------------------------
extern "C" int kv_cache_save(const kv_cache* c, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_save: NULL");
  auto& k = const_cast<kv_cache*>(c)->impl;
  std::lock_guard<std::mutex> g(k.mu);
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_save: cannot open ") + path);
  const int64_t hdr[9] = {(int64_t)kMagicV2, k.L, k.beams, k.H, k.D, k.TS, k.max_tiles, k.num_pages,
                          k.dtype};
  f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  f.write(reinterpret_cast<const char*>(k.h_table.data()), k.entries * sizeof(int32_t));
  std::vector<int64_t> used;
  for (long long p = 0; p < k.num_pages; ++p)
    if (k.refcount[p] > 0) used.push_back(p);
  const int64_t nu = (int64_t)used.size();
  f.write(reinterpret_cast<const char*>(&nu), sizeof(nu));
  for (int64_t p : used) {
    const int32_t p32 = (int32_t)p;
    f.write(reinterpret_cast<const char*>(&p32), sizeof(p32));
  }
  LLM_HIP_RET(hipDeviceSynchronize());
  // per page: K then V, which are adjacent in the pool (one block of 2 pages)
  const size_t blk = k.page_stride();
  const size_t per = std::max<size_t>(1, kStagingBytes / blk);
  std::vector<char> buf;
  PageMover mv;
  for (size_t i0 = 0; i0 < used.size(); i0 += per) {
    const size_t n = std::min(per, used.size() - i0);
    std::vector<int64_t> ids(used.begin() + i0, used.begin() + i0 + n);
    buf.resize(n * blk);
    if (int rc = mv.move(false, buf.data(), static_cast<char*>(k.k_pool), ids, blk, blk)) return rc;
    f.write(buf.data(), buf.size());
  }
  if (!f) return fail(LLM_ERR_IO, "kv_cache_save: write failed");
  return LLM_OK;
}

extern "C" int kv_cache_load(kv_cache* c, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_load: NULL");
  KvCache& k = c->impl;
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_load: cannot open ") + path);
  Snapshot s;
  if (int rc = parse_snapshot(f, path, s)) return rc;  // nothing changed yet
  const int64_t mine[8] = {k.L, k.beams, k.H, k.D, k.TS, k.max_tiles, k.num_pages, k.dtype};
  for (int i = 0; i < 7; ++i)
    if (s.geo[i] != mine[i])
      return fail(LLM_ERR_INVALID, "kv_cache_load: file geometry differs from this cache");
  if (s.geo[7] != mine[7])
    return fail(LLM_ERR_INVALID, "kv_cache_load: file kv_dtype differs from this cache");
  if (int rc = kv_cache_clear(c)) return rc;
  std::unique_lock<std::mutex> g(k.mu);
  k.h_table = s.table;
  k.lru.clear();  // loaded entries are not registered tiles (kv_cache_impl.hpp lru)
  k.lru_pos.clear();
  std::fill(k.refcount.begin(), k.refcount.end(), 0);
  for (int32_t t : k.h_table)
    if (t >= 0) k.refcount[t] += 1;
  k.reset_free_lists();
  LLM_HIP_RET(hipMemcpy(k.d_table, k.h_table.data(), k.entries * sizeof(int32_t),
                        hipMemcpyHostToDevice));
  f.seekg(s.data_off);
  const size_t blk = k.page_stride();
  const size_t per = std::max<size_t>(1, kStagingBytes / blk);
  std::vector<char> buf;
  PageMover mv;
  for (size_t i0 = 0; i0 < s.used.size(); i0 += per) {
    const size_t n = std::min(per, s.used.size() - i0);
    buf.resize(n * blk);
    f.read(buf.data(), buf.size());
    int rc = !f ? fail(LLM_ERR_IO, "kv_cache_load: read failed") : LLM_OK;
    if (!rc) {
      std::vector<int64_t> ids(s.used.begin() + i0, s.used.begin() + i0 + n);
      rc = mv.move(true, buf.data(), static_cast<char*>(k.k_pool), ids, blk, blk);
    }
    if (rc) {  // leave an empty, consistent cache behind
      g.unlock();
      (void)kv_cache_clear(c);
      return rc;
    }
  }
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// reference pool dump: KVTileCache<T>::save_to_file / load_from_file
// ---------------------------------------------------------------------------
extern "C" int kv_cache_save_pools(const kv_cache* c, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_save_pools: NULL");
  auto& k = const_cast<kv_cache*>(c)->impl;
  std::lock_guard<std::mutex> g(k.mu);
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_save_pools: cannot open ") + path);
  LLM_HIP_RET(hipDeviceSynchronize());
  const size_t pb = k.page_bytes();
  const long long per = (long long)std::max<size_t>(1, kStagingBytes / pb);
  std::vector<char> buf;
  PageMover mv;
  for (int kind = 0; kind < 2; ++kind) {  // the whole K pool, then the whole V pool
    char* base = static_cast<char*>(kind ? k.v_pool : k.k_pool);
    for (long long p0 = 0; p0 < k.num_pages; p0 += per) {
      const long long n = std::min(per, k.num_pages - p0);
      std::vector<int64_t> ids((size_t)n);
      for (long long i = 0; i < n; ++i) ids[i] = p0 + i;
      buf.resize((size_t)n * pb);
      if (int rc = mv.move(false, buf.data(), base, ids, pb, k.page_stride())) return rc;
      f.write(buf.data(), buf.size());
    }
  }
  if (!f) return fail(LLM_ERR_IO, "kv_cache_save_pools: write failed");
  return LLM_OK;
}

extern "C" int kv_cache_load_pools(kv_cache* c, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_load_pools: NULL");
  KvCache& k = c->impl;
  std::lock_guard<std::mutex> g(k.mu);
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_load_pools: cannot open ") + path);
  const size_t pb = k.page_bytes();
  const long long want = 2LL * k.num_pages * (long long)pb;
  const long long size = file_size(f);
  uint64_t magic = 0;
  if (size >= 8) {
    f.read(reinterpret_cast<char*>(&magic), sizeof(magic));
    f.seekg(0, std::ios::beg);
  }
  // a page-table snapshot (kv_cache_save; round-1 bindings' default format)
  if (size != want && (magic == kMagic || magic == kMagicV2))
    return fail(LLM_ERR_IO, std::string("kv_cache_load_pools: ") + path +
                                " is a page-table snapshot (APPIMKV), not a pool dump: load it "
                                "with kv_cache_load (KVTileCache.load_from_file(path, "
                                "format='snapshot'))");
  // the reference reads whatever is there (kv_tile_cache.cpp:121-122); a dump
  // of another pool size is refused here before any page changes
  if (size != want)
    return fail(LLM_ERR_IO, std::string("kv_cache_load_pools: ") + path + " holds " +
                                std::to_string(size) + " bytes, this pool dumps to " +
                                std::to_string(want));
  LLM_HIP_RET(hipDeviceSynchronize());
  const long long per = (long long)std::max<size_t>(1, kStagingBytes / pb);
  std::vector<char> buf;
  PageMover mv;
  for (int kind = 0; kind < 2; ++kind) {
    char* base = static_cast<char*>(kind ? k.v_pool : k.k_pool);
    for (long long p0 = 0; p0 < k.num_pages; p0 += per) {
      const long long n = std::min(per, k.num_pages - p0);
      buf.resize((size_t)n * pb);
      f.read(buf.data(), buf.size());
      if (!f) return fail(LLM_ERR_IO, "kv_cache_load_pools: read failed");
      std::vector<int64_t> ids((size_t)n);
      for (long long i = 0; i < n; ++i) ids[i] = p0 + i;
      if (int rc = mv.move(true, buf.data(), base, ids, pb, k.page_stride())) return rc;
    }
  }
  return LLM_OK;
}

// ---------------------------------------------------------------------------
// reference tile records: KVTileCacheCPU<T>::save / load
// ---------------------------------------------------------------------------
extern "C" int kv_cache_save_tiles(const kv_cache* c, int layer, int kind, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_save_tiles: NULL");
  auto& k = const_cast<kv_cache*>(c)->impl;
  LLM_REQUIRE(layer >= 0 && layer < k.L && (kind == 0 || kind == 1),
              "kv_cache_save_tiles: bad layer or kind (0 = K, 1 = V)");
  std::lock_guard<std::mutex> g(k.mu);
  std::vector<int32_t> idx;
  std::vector<int64_t> pages;
  for (int b = 0; b < k.beams; ++b)
    for (int h = 0; h < k.H; ++h)
      for (int t = 0; t < k.max_tiles; ++t) {
        const int32_t p = k.h_table[k.index(layer, b, h, t)];
        if (p < 0) continue;
        idx.insert(idx.end(), {b, h, t});
        pages.push_back(p);
      }
  LLM_REQUIRE(pages.size() <= (size_t)INT32_MAX, "kv_cache_save_tiles: more tiles than an int32 count");
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_save_tiles: cannot open ") + path);
  const int32_t n = (int32_t)pages.size();
  f.write(reinterpret_cast<const char*>(&n), sizeof(n));
  LLM_HIP_RET(hipDeviceSynchronize());
  const size_t pb = k.page_bytes();
  const size_t per = std::max<size_t>(1, kStagingBytes / pb);
  char* base = static_cast<char*>(kind ? k.v_pool : k.k_pool);
  std::vector<char> buf;
  PageMover mv;
  for (size_t i0 = 0; i0 < pages.size(); i0 += per) {
    const size_t m = std::min(per, pages.size() - i0);
    std::vector<int64_t> ids(pages.begin() + i0, pages.begin() + i0 + m);
    buf.resize(m * pb);
    if (int rc = mv.move(false, buf.data(), base, ids, pb, k.page_stride())) return rc;
    for (size_t i = 0; i < m; ++i) {
      f.write(reinterpret_cast<const char*>(&idx[3 * (i0 + i)]), 12);
      f.write(buf.data() + i * pb, pb);
    }
  }
  if (!f) return fail(LLM_ERR_IO, "kv_cache_save_tiles: write failed");
  return LLM_OK;
}

extern "C" int kv_cache_load_tiles(kv_cache* c, int layer, int kind, const char* path) {
  LLM_REQUIRE(c && path, "kv_cache_load_tiles: NULL");
  KvCache& k = c->impl;
  LLM_REQUIRE(layer >= 0 && layer < k.L && (kind == 0 || kind == 1),
              "kv_cache_load_tiles: bad layer or kind (0 = K, 1 = V)");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(LLM_ERR_IO, std::string("kv_cache_load_tiles: cannot open ") + path);
  const size_t pb = k.page_bytes();
  std::vector<int32_t> idx;
  int n = 0;
  if (int rc = parse_tiles(f, path, (long long)pb, &idx, &n)) return rc;
  for (int i = 0; i < n; ++i)
    if (!k.in_range(layer, idx[3 * i], idx[3 * i + 1], idx[3 * i + 2]))
      return fail(LLM_ERR_INVALID, std::string("kv_cache_load_tiles: record ") + std::to_string(i) +
                                       " (" + std::to_string(idx[3 * i]) + ", " +
                                       std::to_string(idx[3 * i + 1]) + ", " +
                                       std::to_string(idx[3 * i + 2]) +
                                       ") is outside this cache's (beam, head, tile) range");
  std::lock_guard<std::mutex> g(k.mu);
  // a later record of the same tile wins (cache_[idx] = data, kv_tile_cache_cpu.cpp:119)
  std::vector<int64_t> pages((size_t)n, -1);
  {
    std::vector<std::pair<size_t, int>> seen;
    seen.reserve(n);
    for (int i = 0; i < n; ++i)
      seen.push_back({k.index(layer, idx[3 * i], idx[3 * i + 1], idx[3 * i + 2]), i});
    std::stable_sort(seen.begin(), seen.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    // the pages the load needs (unmapped tiles, and copy-on-write copies of
    // shared ones, counting each shared page's references down as its tiles
    // are un-shared) must all be free BEFORE anything is allocated: a load that
    // fails leaves the cache unchanged
    long long need = 0;
    {
      std::unordered_map<int32_t, int32_t> refs;
      for (size_t j = 0; j < seen.size(); ++j) {
        if (j + 1 < seen.size() && seen[j + 1].first == seen[j].first) continue;
        const int32_t p = k.h_table[seen[j].first];
        if (p < 0) {  // ensure_tile allocates
          ++need;
          continue;
        }
        auto it = refs.find(p);
        if (it == refs.end()) it = refs.emplace(p, k.refcount[p]).first;
        if (it->second > 1) {
          ++need;
          --it->second;
        }
      }
    }
    if (need > k.free_count())
      return fail(LLM_ERR_OOM, "kv_cache_load_tiles: the load needs " + std::to_string(need) +
                                   " free pages, the pool has " + std::to_string(k.free_count()) +
                                   " (cache unchanged)");
    for (size_t j = 0; j < seen.size(); ++j) {
      if (j + 1 < seen.size() && seen[j + 1].first == seen[j].first) continue;  // superseded
      const int i = seen[j].second;
      int32_t p;
      if (int rc = k.ensure_tile(layer, idx[3 * i], idx[3 * i + 1], idx[3 * i + 2], true, &p))
        return rc;
      pages[i] = p;
    }
  }
  if (int rc = k.sync(nullptr)) return rc;  // copy-on-write copies, table entries
  LLM_HIP_RET(hipDeviceSynchronize());
  const size_t per = std::max<size_t>(1, kStagingBytes / pb);
  char* base = static_cast<char*>(kind ? k.v_pool : k.k_pool);
  std::vector<char> buf;
  PageMover mv;
  for (size_t i0 = 0; i0 < (size_t)n; i0 += per) {
    const size_t m = std::min(per, (size_t)n - i0);
    buf.resize(m * pb);
    for (size_t i = 0; i < m; ++i) {
      f.seekg(4 + (long long)(i0 + i) * (12 + (long long)pb) + 12);
      f.read(buf.data() + i * pb, pb);
    }
    if (!f) return fail(LLM_ERR_IO, "kv_cache_load_tiles: read failed");
    std::vector<int64_t> ids(pages.begin() + i0, pages.begin() + i0 + m);
    if (int rc = mv.move(true, buf.data(), base, ids, pb, k.page_stride())) return rc;
  }
  return LLM_OK;
}
