"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's two KV-cache file formats, used by the
tests as the checker of the build's kv_cache_{save,load}_{tiles,pools}:

* ``KVTileCacheCPU<T>::save`` / ``load`` (kv_cache/kv_tile_cache_cpu.cpp:89-123):
  ``int32 count``, then per tile the 12-byte ``TileIndex {int batch_id, head_id,
  tile_id}`` (kv_tile_cache_cpu.hpp:14-18, written raw at :99) followed by
  ``tile_size_`` elements of ``T`` (:100).  Record order is the iteration order
  of the reference's ``unordered_map`` (:98), i.e. unspecified; on load a later
  record of the same index replaces an earlier one (``cache_[idx] = ...``, :119).
  Pinned by the reference-built fixtures ``tests/golden/kvtiles_*.npz``.
* ``KVTileCache<T>::save_to_file`` / ``load_from_file``
  (kv_cache/kv_tile_cache.cpp:105-125): the raw K pool
  ``[total_pages][tile_size][head_dim]`` then the raw V pool, no header.  That
  file cannot be produced by the reference here (CUDA); the layout is
  restated from :108-113.
"""
from __future__ import annotations

import numpy as np

_IDX = np.dtype([("batch_id", "<i4"), ("head_id", "<i4"), ("tile_id", "<i4")])


def read_tiles(data: bytes, tile_elems: int, dtype) -> list[tuple[tuple[int, int, int], np.ndarray]]:
    """Records of a KVTileCacheCPU save file, in file order (kv_tile_cache_cpu.cpp:106-123)."""
    dtype = np.dtype(dtype)
    buf = memoryview(data)
    (count,) = np.frombuffer(buf[:4], "<i4")
    rec = 12 + tile_elems * dtype.itemsize
    if count < 0 or len(buf) != 4 + int(count) * rec:
        raise ValueError(f"tile file: {len(buf)} bytes for {count} records of {rec}")
    out = []
    for i in range(int(count)):
        off = 4 + i * rec
        b, h, t = (int(x) for x in np.frombuffer(buf[off:off + 12], "<i4"))
        tile = np.frombuffer(buf[off + 12:off + rec], dtype).copy()
        out.append(((b, h, t), tile))
    return out


def write_tiles(records) -> bytes:
    """KVTileCacheCPU::save (kv_tile_cache_cpu.cpp:90-102) for records given in
    the order they are to be written: [((batch, head, tile), tile_array), ...]."""
    parts = [np.int32(len(records)).tobytes()]
    for (b, h, t), tile in records:
        parts.append(np.array([b, h, t], "<i4").tobytes())
        parts.append(np.ascontiguousarray(tile).tobytes())
    return b"".join(parts)


def tiles_dict(records) -> dict:
    """index -> tile after a load: later records win (kv_tile_cache_cpu.cpp:119)."""
    d = {}
    for idx, tile in records:
        d[idx] = tile
    return d


def pool_dump(k_pool: np.ndarray, v_pool: np.ndarray) -> bytes:
    """KVTileCache::save_to_file (kv_tile_cache.cpp:106-114): K pool bytes then V
    pool bytes, each [total_pages][tile_size][head_dim] of T."""
    assert k_pool.shape == v_pool.shape and k_pool.dtype == v_pool.dtype
    return np.ascontiguousarray(k_pool).tobytes() + np.ascontiguousarray(v_pool).tobytes()


def pool_load(data: bytes, pages: int, tile_size: int, head_dim: int, dtype):
    """KVTileCache::load_from_file (kv_tile_cache.cpp:117-125) -> (k_pool, v_pool)."""
    dtype = np.dtype(dtype)
    n = pages * tile_size * head_dim
    a = np.frombuffer(data, dtype, count=2 * n)
    return a[:n].reshape(pages, tile_size, head_dim), a[n:].reshape(pages, tile_size, head_dim)
