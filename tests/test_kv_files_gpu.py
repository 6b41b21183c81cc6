"""The reference's KV-cache files through the build's cache (GPU).

* KVTileCacheCPU<T>::save / load (kv_cache/kv_tile_cache_cpu.cpp:89-123): the
  reference-built record files (tests/golden/kvtiles_*.npz) load into the page
  pools bit for bit, attention over the loaded pages matches the oracle, and the
  build's save writes the same records byte for byte (record order aside: the
  reference's order is its hash map's).
* KVTileCache<T>::save_to_file / load_from_file (kv_cache/kv_tile_cache.cpp:
  105-125): raw K pool then raw V pool, checked against the oracle's
  restatement (oracle/kv_formats.py) and round-tripped.
* Refused files leave the cache as it was.
"""
import ctypes

import numpy as np
import pytest

from oracle import kv_formats
from _util import assert_parity, GOLDEN, rel_err

pytestmark = pytest.mark.gpu

DTYPE = {np.dtype(np.float16): "float16", np.dtype(np.float32): "float32",
         np.dtype(np.int8): "int8"}


def _fixture(name):
    f = np.load(GOLDEN / f"kvtiles_{name}.npz")
    return {k: f[k] for k in f.files}


def _pools(kv, num_pages, ts, D, dtype):
    """(K pool, V pool) [num_pages][ts][D] read back from the device."""
    import torch
    v = kv.view(0)
    tdt = {np.dtype(np.float16): torch.int16, np.dtype(np.float32): torch.float32,
           np.dtype(np.int8): torch.int8}[np.dtype(dtype)]
    t = torch.empty(num_pages * 2 * ts * D, dtype=tdt, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(v["k_pool"]),
                         t.numel() * t.element_size(), 3) == 0
    both = t.cpu().numpy().view(np.dtype(dtype)).reshape(num_pages, 2, ts, D)
    return both[:, 0].copy(), both[:, 1].copy()


def _cache(ts, D, dtype, beams=4, H=2, max_tiles=6, pages=40):
    import llm_decoder
    kv = llm_decoder.KVTileCache()
    kv.init(num_pages=pages, tile_size=ts, head_dim=D, num_layers=1, num_beams=beams,
            num_heads=H, max_tiles=max_tiles, dtype=DTYPE[np.dtype(dtype)])
    return kv


@pytest.mark.parametrize("name", ["f16_ts16_d64", "f32_ts16_d32", "i8_ts32_d64"])
def test_reference_tile_files_load_and_save(gpu, tmp_path, name):
    f = _fixture(name)
    data, idx, ts, D = f["data"], f["idx"], int(f["ts"]), int(f["D"])
    ref_path = tmp_path / "ref_k.bin"
    ref_path.write_bytes(f["file_bytes"].tobytes())
    kv = _cache(ts, D, data.dtype)
    kv.load_tiles(str(ref_path), "k")
    kv.sync_page_table_to_gpu()
    kpool, vpool = _pools(kv, 40, ts, D, data.dtype)
    pages = set()
    for (b, h, t), tile in zip(idx, data):
        p = kv.lookup(int(b), int(h), int(t))
        assert p >= 0
        pages.add(p)
        assert kpool[p].tobytes() == tile.tobytes()  # bit for bit
    assert len(pages) == len(idx) and kv.free_pages() == 40 - len(idx)
    # the build's save: the same records, each byte for byte, in (beam, head, tile) order
    out = tmp_path / "ours_k.bin"
    kv.save_tiles(str(out), "k")
    raw = out.read_bytes()
    recs = kv_formats.read_tiles(raw, ts * D, data.dtype)
    assert [r[0] for r in recs] == sorted(tuple(int(x) for x in i) for i in idx)
    ref_recs = kv_formats.read_tiles(f["file_bytes"].tobytes(), ts * D, data.dtype)
    assert raw == kv_formats.write_tiles(sorted(ref_recs, key=lambda r: r[0]))
    # V tiles go to the V half of the same pages
    kv.load_tiles(str(ref_path), "v")
    _, vpool = _pools(kv, 40, ts, D, data.dtype)
    for (b, h, t), tile in zip(idx, data):
        assert vpool[kv.lookup(int(b), int(h), int(t))].tobytes() == tile.tobytes()
    assert kv.free_pages() == 40 - len(idx)


def test_attention_over_reference_tile_files(gpu, oracle, tmp_path):
    """Pages loaded from the reference's K and V record files feed paged
    attention; unmapped tiles are missing pages (masked), as in the oracle."""
    import torch
    import llm_decoder
    rng = np.random.default_rng(11)
    B, H, D, ts, nt = 3, 2, 64, 16, 4
    T = nt * ts - 5
    present = rng.random((B, H, nt)) < 0.8
    present[:, :, 0] = True
    recs_k, recs_v = [], []
    kt = rng.standard_normal((B, H, nt, ts, D)).astype(np.float16) * np.float16(D ** -0.25)
    vt = rng.standard_normal((B, H, nt, ts, D)).astype(np.float16)
    order = [(b, h, t) for b in range(B) for h in range(H) for t in range(nt) if present[b, h, t]]
    rng.shuffle(order)  # the reference writes in hash-map order: any order must load
    for (b, h, t) in order:
        recs_k.append(((b, h, t), kt[b, h, t]))
        recs_v.append(((b, h, t), vt[b, h, t]))
    (tmp_path / "k.bin").write_bytes(kv_formats.write_tiles(recs_k))
    (tmp_path / "v.bin").write_bytes(kv_formats.write_tiles(recs_v))
    kv = _cache(ts, D, np.float16, beams=B, H=H, max_tiles=nt, pages=64)
    kv.load_tiles(str(tmp_path / "k.bin"), "k")
    kv.load_tiles(str(tmp_path / "v.bin"), "v")
    kv.sync_page_table_to_gpu()
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    qd = torch.from_numpy(q).cuda()
    out = torch.empty((B, H, D), device="cuda")
    ws_bytes = llm_decoder.workspace_bytes(B, H, D, nt)
    ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device="cuda")
    llm_decoder.paged_attention(kv.handle, 0, qd.data_ptr(), out.data_ptr(), B=B, H=H, D=D, T=T,
                                workspace=ws.data_ptr(), workspace_bytes=ws_bytes)
    torch.cuda.synchronize()
    kpool = np.zeros((B * H * nt, ts, D), np.float32)
    vpool = np.zeros_like(kpool)
    pt = np.full((B, H, nt), -1, np.int32)
    for i, (b, h, t) in enumerate(order):
        pt[b, h, t] = i
        kpool[i], vpool[i] = kt[b, h, t], vt[b, h, t]
    ref = oracle.paged_attention(q, kpool, vpool, pt, T=T)
    assert_parity(out.cpu().numpy(), ref, 1e-3)


def test_tile_load_semantics_cow_duplicates_and_refusals(gpu, tmp_path):
    """A record for a tile shared with a forked beam is copied-on-write; a later
    record of the same tile wins (kv_tile_cache_cpu.cpp:119); a record outside
    the cache's range, or a short file, is refused with the cache unchanged."""
    ts, D = 16, 64
    rng = np.random.default_rng(5)
    kv = _cache(ts, D, np.float16, beams=4, H=2, max_tiles=6, pages=40)
    base = [((0, h, t), rng.standard_normal((ts, D)).astype(np.float16))
            for h in range(2) for t in range(2)]
    (tmp_path / "base.bin").write_bytes(kv_formats.write_tiles(base))
    kv.load_tiles(str(tmp_path / "base.bin"), "k")
    kv.fork(0, 3)
    shared = kv.lookup(0, 1, 1)
    assert kv.lookup(3, 1, 1) == shared and kv.free_pages() == 36
    a = rng.standard_normal((ts, D)).astype(np.float16)
    b = rng.standard_normal((ts, D)).astype(np.float16)
    (tmp_path / "upd.bin").write_bytes(kv_formats.write_tiles([((3, 1, 1), a), ((3, 1, 1), b)]))
    kv.load_tiles(str(tmp_path / "upd.bin"), "k")
    kv.sync_page_table_to_gpu()
    own = kv.lookup(3, 1, 1)
    assert own not in (-1, shared) and kv.lookup(0, 1, 1) == shared and kv.free_pages() == 35
    kpool, _ = _pools(kv, 40, ts, D, np.float16)
    assert kpool[own].tobytes() == b.tobytes()            # the later record won
    assert kpool[shared].tobytes() == base[3][1].tobytes()  # beam 0 untouched
    before = kv.free_pages()
    for bad in ([((4, 0, 0), a)], [((0, 2, 0), a)], [((0, 0, 6), a)]):  # beam / head / tile
        (tmp_path / "bad.bin").write_bytes(kv_formats.write_tiles(bad))
        with pytest.raises(RuntimeError, match="outside"):
            kv.load_tiles(str(tmp_path / "bad.bin"), "k")
    (tmp_path / "short.bin").write_bytes(kv_formats.write_tiles([((1, 0, 0), a)])[:-2])
    with pytest.raises(RuntimeError, match="bytes"):
        kv.load_tiles(str(tmp_path / "short.bin"), "k")
    assert kv.free_pages() == before and kv.lookup(1, 0, 0) == -1
    with pytest.raises(ValueError):
        kv.load_tiles(str(tmp_path / "base.bin"), "x")


@pytest.mark.parametrize("dtype", [np.float16, np.float32])
def test_reference_pool_dump_round_trip(gpu, tmp_path, dtype):
    """save_to_file writes KVTileCache's dump (K pool then V pool, no header);
    load_from_file restores the pools and keeps the reader's page table."""
    ts, D, pages = 16, 32, 24
    rng = np.random.default_rng(9)
    kv = _cache(ts, D, dtype, beams=2, H=2, max_tiles=4, pages=pages)
    recs = [((b, h, t), rng.standard_normal((ts, D)).astype(dtype))
            for b in range(2) for h in range(2) for t in range(3)]
    (tmp_path / "k.bin").write_bytes(kv_formats.write_tiles(recs))
    (tmp_path / "v.bin").write_bytes(kv_formats.write_tiles([(i, -x) for i, x in recs]))
    kv.load_tiles(str(tmp_path / "k.bin"), "k")
    kv.load_tiles(str(tmp_path / "v.bin"), "v")
    kpool, vpool = _pools(kv, pages, ts, D, dtype)
    path = tmp_path / "pools.bin"
    kv.save_to_file(str(path))  # default: the reference's format
    raw = path.read_bytes()
    assert raw == kv_formats.pool_dump(kpool, vpool)
    assert len(raw) == 2 * pages * ts * D * np.dtype(dtype).itemsize
    kv2 = _cache(ts, D, dtype, beams=2, H=2, max_tiles=4, pages=pages)
    kv2.load_from_file(str(path))
    k2, v2 = _pools(kv2, pages, ts, D, dtype)
    assert k2.tobytes() == kpool.tobytes() and v2.tobytes() == vpool.tobytes()
    assert kv2.lookup(0, 0, 0) == -1 and kv2.free_pages() == pages  # table not in the file
    k_ref, v_ref = kv_formats.pool_load(raw, pages, ts, D, dtype)
    assert k_ref.tobytes() == kpool.tobytes() and v_ref.tobytes() == vpool.tobytes()
    # a dump of another pool size is refused before any page changes
    small = _cache(ts, D, dtype, beams=2, H=2, max_tiles=4, pages=pages - 1)
    with pytest.raises(RuntimeError, match="bytes"):
        small.load_from_file(str(path))
    (tmp_path / "cut.bin").write_bytes(raw[:-4])
    with pytest.raises(RuntimeError, match="bytes"):
        kv2.load_from_file(str(tmp_path / "cut.bin"))
    k3, _ = _pools(kv2, pages, ts, D, dtype)
    assert k3.tobytes() == kpool.tobytes()


def test_corrupt_snapshot_leaves_cache_unchanged(gpu, tmp_path):
    """kv_cache_load validates the whole snapshot before it changes the cache
    (ids outside the pool, truncation)."""
    ts, D = 16, 64
    rng = np.random.default_rng(2)
    kv = _cache(ts, D, np.float16, beams=2, H=2, max_tiles=4, pages=20)
    recs = [((b, 0, t), rng.standard_normal((ts, D)).astype(np.float16))
            for b in range(2) for t in range(2)]
    (tmp_path / "k.bin").write_bytes(kv_formats.write_tiles(recs))
    kv.load_tiles(str(tmp_path / "k.bin"), "k")
    snap = tmp_path / "snap.bin"
    kv.save_to_file(str(snap), format="snapshot")
    raw = bytearray(snap.read_bytes())
    table_off = 72
    bad_table = bytearray(raw)
    bad_table[table_off:table_off + 4] = np.int32(20).tobytes()  # page 20 of 20
    dest = _cache(ts, D, np.float16, beams=2, H=2, max_tiles=4, pages=20)
    dest.load_tiles(str(tmp_path / "k.bin"), "k")
    before = [dest.lookup(b, 0, t) for b in range(2) for t in range(4)]
    for blob in (bytes(bad_table), bytes(raw[:-1]), bytes(raw[:100])):
        (tmp_path / "bad.bin").write_bytes(blob)
        with pytest.raises(RuntimeError):
            dest.load_from_file(str(tmp_path / "bad.bin"), format="snapshot")
        assert [dest.lookup(b, 0, t) for b in range(2) for t in range(4)] == before
        assert dest.free_pages() == 16
    dest.load_from_file(str(snap), format="snapshot")
    assert [dest.lookup(b, 0, t) for b in range(2) for t in range(4)] == \
        [kv.lookup(b, 0, t) for b in range(2) for t in range(4)]


def test_tile_load_out_of_pages_leaves_cache_unchanged(gpu, tmp_path):
    """A record file that needs more free pages (new tiles plus copy-on-write
    copies of forked ones) than the pool has is refused before any page is
    allocated: the page table and the free count stay as they were."""
    ts, D = 16, 64
    rng = np.random.default_rng(8)
    kv = _cache(ts, D, np.float16, beams=4, H=2, max_tiles=6, pages=12)
    base = [((0, h, t), rng.standard_normal((ts, D)).astype(np.float16))
            for h in range(2) for t in range(3)]
    (tmp_path / "base.bin").write_bytes(kv_formats.write_tiles(base))
    kv.load_tiles(str(tmp_path / "base.bin"), "k")
    kv.fork(0, 1)  # 6 shared pages
    assert kv.free_pages() == 6
    before = [kv.lookup(b, h, t) for b in range(4) for h in range(2) for t in range(6)]
    # 4 copies-on-write of beam 1's shared tiles + 3 new tiles = 7 > 6 free
    recs = [((1, h, t), rng.standard_normal((ts, D)).astype(np.float16))
            for h in range(2) for t in range(2)]
    recs += [((2, 0, t), rng.standard_normal((ts, D)).astype(np.float16)) for t in range(3)]
    (tmp_path / "big.bin").write_bytes(kv_formats.write_tiles(recs))
    with pytest.raises(RuntimeError, match="free pages"):
        kv.load_tiles(str(tmp_path / "big.bin"), "k")
    assert [kv.lookup(b, h, t) for b in range(4) for h in range(2) for t in range(6)] == before
    assert kv.free_pages() == 6
    # one record fewer fits exactly (6 pages) and loads
    (tmp_path / "fit.bin").write_bytes(kv_formats.write_tiles(recs[:-1]))
    kv.load_tiles(str(tmp_path / "fit.bin"), "k")
    assert kv.free_pages() == 0 and kv.lookup(1, 0, 0) != kv.lookup(0, 0, 0)


def test_pool_load_of_a_snapshot_names_the_format(gpu, tmp_path):
    """load_from_file's default format is the reference's pool dump; given a
    page-table snapshot (the round-1 default) it says so instead of failing on
    the size alone."""
    ts, D = 16, 64
    kv = _cache(ts, D, np.float16, beams=2, H=2, max_tiles=4, pages=20)
    snap = tmp_path / "snap.bin"
    kv.save_to_file(str(snap), format="snapshot")
    with pytest.raises(RuntimeError, match="format='snapshot'"):
        kv.load_from_file(str(snap))
    kv.load_from_file(str(snap), format="snapshot")
