"""KV page cache / page table (kv_cache/page_table.hpp:5-37,
kv_cache/kv_tile_cache.hpp:9-41 semantics) through the C ABI and the pybind11
classes: index arithmetic bit-exact against the oracle, free-list allocation,
beam fork with copy-on-write, save/load, and attention over a forked cache."""
import ctypes

import numpy as np
import pytest

from _util import assert_parity, rel_err

pytestmark = pytest.mark.gpu


def test_page_table_semantics(gpu, oracle):
    import torch
    import llm_decoder
    pt = llm_decoder.PageTable()
    pt.init(2, 3, 5)
    assert pt.lookup(0, 0, 0) == -1  # init to -1 (page_table.cpp:22-25)
    pt.assign(1, 2, 4, 7)
    pt.assign(0, 1, 3, 2)
    assert pt.lookup(1, 2, 4) == 7 and pt.lookup(0, 1, 3) == 2
    assert pt.lookup(2, 0, 0) == -1 and pt.lookup(0, 3, 0) == -1  # out of range -> -1
    pt.remove(1, 2, 4)
    pt.sync_to_gpu()
    torch.cuda.synchronize()
    # device copy equals the host mirror (single source of truth); index
    # = beam*(H*NT) + head*NT + tile (page_table.hpp:41)
    host = np.full(30, -1, np.int32)
    host[0 * 15 + 1 * 5 + 3] = 2
    hip_ptr = pt.device_data()
    arr = (ctypes.c_int32 * 30)()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(ctypes.addressof(arr), ctypes.c_void_p(hip_ptr), 120, 2) == 0
    np.testing.assert_array_equal(np.frombuffer(arr, np.int32), host)
    pt.clear()
    assert pt.lookup(0, 1, 3) == -1


def test_kv_cache_alloc_fork_cow(gpu):
    import llm_capi
    lib = llm_capi.load()
    h = ctypes.c_void_p()
    llm_capi.check(lib.kv_cache_create(2, 3, 2, 64, 16, 8, 40, ctypes.byref(h)))
    try:
        assert lib.kv_cache_free_pages(h) == 40
        llm_capi.check(lib.kv_cache_reserve(h, 0, 33))  # 3 tiles x 2 heads x 2 layers
        assert lib.kv_cache_free_pages(h) == 40 - 12
        pages = {lib.kv_cache_lookup(h, l, 0, hh, t) for l in range(2) for hh in range(2) for t in range(3)}
        assert len(pages) == 12 and -1 not in pages  # distinct ids (no map.size() aliasing)
        llm_capi.check(lib.kv_cache_fork(h, 0, 1))
        assert lib.kv_cache_free_pages(h) == 40 - 12  # shared, not copied
        assert lib.kv_cache_lookup(h, 1, 1, 1, 2) == lib.kv_cache_lookup(h, 1, 0, 1, 2)
        # writing into beam 1's shared last tile copies it first (copy-on-write)
        k = np.ones((1, 2, 64), np.float16).view(np.uint16)
        llm_capi.check(lib.kv_cache_write_tokens(h, 0, 1, 33, 1, k.ctypes.data, k.ctypes.data))
        assert lib.kv_cache_lookup(h, 0, 1, 0, 2) != lib.kv_cache_lookup(h, 0, 0, 0, 2)
        assert lib.kv_cache_lookup(h, 1, 1, 0, 2) == lib.kv_cache_lookup(h, 1, 0, 0, 2)  # other layer still shared
        assert lib.kv_cache_free_pages(h) == 40 - 12 - 2
        llm_capi.check(lib.kv_cache_release(h, 0))
        assert lib.kv_cache_free_pages(h) == 40 - 12 - 2 + 2  # only pages no other beam holds
        llm_capi.check(lib.kv_cache_release(h, 1))
        assert lib.kv_cache_free_pages(h) == 40
        # exhaustion is an error, not a silent eviction
        llm_capi.check(lib.kv_cache_reserve(h, 2, 16 * 8))  # 32 of 40 pages
        assert lib.kv_cache_reserve(h, 0, 16 * 8) == llm_capi.LLM_ERR_OOM
    finally:
        lib.kv_cache_destroy(h)


class _RefLru:
    """KVTileCache<T>::register_tile / update_lru / evict_if_needed
    (kv_cache/kv_tile_cache.cpp:64-98) restated over tile keys: which tiles
    hold a page, and the recency order (most recent first).  The reference's
    page ids (map.size(), kv_tile_cache.cpp:71) alias live pages after an
    eviction, so page ids are not compared -- only which tiles are mapped."""

    def __init__(self, total):
        self.total, self.mapped, self.lru = total, set(), []

    def register(self, key):
        if key not in self.mapped:
            if len(self.mapped) >= self.total:  # evict_if_needed
                self.mapped.discard(self.lru.pop())
            self.mapped.add(key)
        if key in self.lru:  # update_lru
            self.lru.remove(key)
        self.lru.insert(0, key)


def test_kv_cache_lru_eviction_vs_reference(gpu):
    """kv_cache_set_eviction(LLM_EVICT_LRU): a random stream of register_tile
    calls over more tiles than the pool holds keeps exactly the reference's
    set of mapped tiles after every call, on distinct pages; the default
    policy reports LLM_ERR_OOM and changes nothing; kv_cache_clear resets the
    recency list; the pybind KVTileCache.set_eviction drives the same path."""
    import llm_capi
    lib = llm_capi.load()
    pages = 6
    h = ctypes.c_void_p()
    llm_capi.check(lib.kv_cache_create(2, 2, 2, 64, 16, 8, pages, ctypes.byref(h)))
    try:
        keys = [(l, b, hh, t) for l in range(2) for b in range(2) for hh in range(2) for t in range(8)]
        page = ctypes.c_int32()
        for k in keys[:pages]:
            llm_capi.check(lib.kv_cache_register_tile(h, *k, ctypes.byref(page)))
        # default policy: the pool is full -> OOM, no entry touched
        before = [lib.kv_cache_lookup(h, *k) for k in keys]
        assert lib.kv_cache_register_tile(h, *keys[pages], ctypes.byref(page)) == llm_capi.LLM_ERR_OOM
        assert [lib.kv_cache_lookup(h, *k) for k in keys] == before
        llm_capi.check(lib.kv_cache_clear(h))
        llm_capi.check(lib.kv_cache_set_eviction(h, llm_capi.LLM_EVICT_LRU))
        assert lib.kv_cache_set_eviction(h, 7) == llm_capi.LLM_ERR_INVALID
        ref = _RefLru(pages)
        rng = np.random.default_rng(3)
        pool = keys[:10]  # 10 tiles competing for 6 pages: hits and evictions
        for i in range(300):
            k = pool[int(rng.integers(len(pool)))]
            llm_capi.check(lib.kv_cache_register_tile(h, *k, ctypes.byref(page)))
            ref.register(k)
            got = {kk: lib.kv_cache_lookup(h, *kk) for kk in pool}
            mapped = {kk for kk, p in got.items() if p >= 0}
            assert mapped == ref.mapped, (i, k, sorted(mapped ^ ref.mapped))
            assert got[k] == page.value and 0 <= page.value < pages
            assert len({got[kk] for kk in mapped}) == len(mapped)  # distinct pages
            assert lib.kv_cache_free_pages(h) == pages - len(mapped)
        # a page a forked beam shares is never evicted for nothing: beam 1 of
        # layer 0 shares beam 0's pages, so only unshared entries can go
        llm_capi.check(lib.kv_cache_clear(h))
        for t in range(3):
            llm_capi.check(lib.kv_cache_register_tile(h, 0, 0, 0, t, ctypes.byref(page)))
        llm_capi.check(lib.kv_cache_fork(h, 0, 1))  # beam 1 := beam 0 (both layers)
        for t in range(3, 6):
            llm_capi.check(lib.kv_cache_register_tile(h, 1, 0, 0, t, ctypes.byref(page)))
        # pool full (3 shared + 3 own); the LRU entries 0..2 are shared: the
        # next tile evicts layer 1's tile 3, the oldest unshared one
        llm_capi.check(lib.kv_cache_register_tile(h, 1, 0, 1, 0, ctypes.byref(page)))
        assert lib.kv_cache_lookup(h, 1, 0, 0, 3) == -1
        assert all(lib.kv_cache_lookup(h, 0, 0, 0, t) >= 0 for t in range(3))
        assert all(lib.kv_cache_lookup(h, 0, 1, 0, t) == lib.kv_cache_lookup(h, 0, 0, 0, t)
                   for t in range(3))
        # releasing beam 1 leaves layer 0's tiles 0..2 unshared again, so the
        # next eviction takes tile 0, now the oldest evictable entry
        llm_capi.check(lib.kv_cache_release(h, 1))
        llm_capi.check(lib.kv_cache_register_tile(h, 1, 1, 1, 1, ctypes.byref(page)))
        assert lib.kv_cache_lookup(h, 0, 0, 0, 0) == -1  # now the oldest, unshared
        # an entry another call rewrites leaves the recency list: register beam
        # 0's tiles, release the beam, let the decoder's reserve put pages back
        # on the same (layer, beam, head, tile) entries, then fill the pool by
        # register_tile -- the eviction must take a registered tile, never a
        # reserved one (a stale list entry used to evict it)
        llm_capi.check(lib.kv_cache_clear(h))
        for t in range(3):
            llm_capi.check(lib.kv_cache_register_tile(h, 0, 0, 0, t, ctypes.byref(page)))
        llm_capi.check(lib.kv_cache_release(h, 0))
        llm_capi.check(lib.kv_cache_reserve(h, 0, 16))  # tile 0 of beam 0: 2 layers x 2 heads
        reserved = {(l, 0, hh, 0): lib.kv_cache_lookup(h, l, 0, hh, 0) for l in range(2) for hh in range(2)}
        assert all(p >= 0 for p in reserved.values())
        for t in range(2):
            llm_capi.check(lib.kv_cache_register_tile(h, 1, 1, 0, t, ctypes.byref(page)))
        assert lib.kv_cache_free_pages(h) == 0
        llm_capi.check(lib.kv_cache_register_tile(h, 1, 1, 0, 2, ctypes.byref(page)))
        assert lib.kv_cache_lookup(h, 1, 1, 0, 0) == -1  # the least recently registered
        assert {k: lib.kv_cache_lookup(h, *k) for k in reserved} == reserved
        # kv_cache_assign / kv_cache_remove rewrite entries too: a registered
        # tile re-assigned by hand is no longer an eviction candidate
        llm_capi.check(lib.kv_cache_assign(h, 1, 1, 0, 1, lib.kv_cache_lookup(h, 1, 1, 0, 1)))
        p_assigned = lib.kv_cache_lookup(h, 1, 1, 0, 1)
        llm_capi.check(lib.kv_cache_remove(h, 1, 1, 0, 2))
        llm_capi.check(lib.kv_cache_register_tile(h, 1, 1, 1, 0, ctypes.byref(page)))  # free page
        assert lib.kv_cache_register_tile(h, 1, 1, 1, 1, ctypes.byref(page)) == llm_capi.LLM_OK
        assert lib.kv_cache_lookup(h, 1, 1, 1, 0) == -1  # the only registered entry left
        assert lib.kv_cache_lookup(h, 1, 1, 0, 1) == p_assigned
        assert {k: lib.kv_cache_lookup(h, *k) for k in reserved} == reserved
    finally:
        lib.kv_cache_destroy(h)
    # the pybind KVTileCache (kv_tile_cache.hpp:9-41 names)
    import llm_decoder
    c = llm_decoder.KVTileCache()
    c.init(3, 16, 64, 1, 1, 1, 8, "float16")
    with pytest.raises(RuntimeError):
        for t in range(4):
            c.register_tile(0, 0, t, 0)
    c.set_eviction("lru")
    p3 = c.register_tile(0, 0, 3, 0)  # evicts tile 0, the least recently registered
    assert c.lookup(0, 0, 0, 0) == -1 and p3 >= 0
    with pytest.raises(ValueError):
        c.set_eviction("fifo")


def test_forked_beams_attention_and_save_load(gpu, oracle, tmp_path):
    """Beams forked from a shared prefix, then diverging tokens written with
    COW; pa_decode over the cache (beam_ids routing) matches the oracle on the
    pools read back; save/load round-trips the cache bit-exactly."""
    import torch
    import llm_capi
    import llm_decoder
    rng = np.random.default_rng(3)
    H, D, TS, prefix, tail, beams = 2, 128, 16, 40, 9, 3
    kv = llm_decoder.KVTileCache()
    kv.init(num_pages=64, tile_size=TS, head_dim=D, num_layers=1, num_beams=beams,
            num_heads=H, max_tiles=8)
    kp = rng.standard_normal((prefix, H, D)).astype(np.float16)
    vp = rng.standard_normal((prefix, H, D)).astype(np.float16)
    kv.write_tokens(0, 0, 0, kp.view(np.uint16), vp.view(np.uint16))
    for b in (1, 2):
        kv.fork(0, b)
    tails = {}
    for b in range(beams):
        kt = rng.standard_normal((tail, H, D)).astype(np.float16)
        vt = rng.standard_normal((tail, H, D)).astype(np.float16)
        kv.write_tokens(0, b, prefix, kt.view(np.uint16), vt.view(np.uint16))
        tails[b] = (kt, vt)
    T = prefix + tail
    view = kv.view(0)
    num_pages = view["num_pages"]
    lib = llm_capi.load()
    # read back pools and table through torch
    def dev_copy(ptr, n, dtype):
        t = torch.empty(n, dtype=dtype, device="cuda")
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr),
                             n * t.element_size(), 3) == 0
        return t
    # K and V pages interleave in one allocation: [num_pages][K page | V page]
    assert view["page_stride"] == 2 * TS * D * 2
    assert view["v_pool"] == view["k_pool"] + TS * D * 2
    both = dev_copy(view["k_pool"], num_pages * 2 * TS * D, torch.float16).reshape(num_pages, 2, TS, D)
    kpool, vpool = both[:, 0], both[:, 1]
    table = dev_copy(view["page_table"], beams * H * 8, torch.int32).reshape(beams, H, 8)
    # the pools hold exactly what was written, per beam
    for b in range(beams):
        for t in range(T):
            page = kv.lookup(b, 1, t // TS)
            want = kp[t, 1] if t < prefix else tails[b][0][t - prefix, 1]
            np.testing.assert_array_equal(kpool[page, t % TS].cpu().numpy(), want)
    q = (rng.standard_normal((4, H, D)) * D ** -0.25).astype(np.float32)
    beam_ids = np.array([2, 0, 1, 2], np.int32)
    out = llm_capi.pa_decode(torch.from_numpy(q).cuda(), kpool, vpool, table, T=T,
                             beam_ids=torch.from_numpy(beam_ids).cuda()).cpu().numpy()
    ref = oracle.paged_attention(q, kpool.float().cpu().numpy(), vpool.float().cpu().numpy(),
                                 table.cpu().numpy(), T=T, beam_ids=beam_ids)
    assert_parity(out, ref, 1e-3)
    # beam-aware schedule (rows in groups of 2 and 4): group 2 is bitwise the
    # plain schedule; group 4 may place its split boundaries by cost (shared
    # prefix vs private tail), which changes only the fp32 merge rounding
    for g in (2, 4):
        outg = llm_capi.pa_decode(torch.from_numpy(q).cuda(), kpool, vpool, table, T=T,
                                  beam_ids=torch.from_numpy(beam_ids).cuda(),
                                  row_group=g).cpu().numpy()
        if g == 2:
            np.testing.assert_array_equal(outg, out)
        else:
            assert rel_err(outg, out) < 1e-5
    # save / load round trip
    path = str(tmp_path / "kv.bin")
    kv.save_to_file(path, format="snapshot")
    kv2 = llm_decoder.KVTileCache()
    kv2.init(num_pages=64, tile_size=TS, head_dim=D, num_layers=1, num_beams=beams,
             num_heads=H, max_tiles=8)
    kv2.load_from_file(path, format="snapshot")
    for b in range(beams):
        for t in range(4):
            assert kv2.lookup(b, 0, t) == kv.lookup(b, 0, t)
    v2 = kv2.view(0)
    kpool2 = dev_copy(v2["k_pool"], num_pages * 2 * TS * D,
                      torch.float16).reshape(num_pages, 2, TS, D)[:, 0]
    used = sorted({kv.lookup(b, h, t) for b in range(beams) for h in range(H) for t in range(4)})
    # bitwise (rows past the written tokens are never-written bits, possibly NaN)
    assert torch.equal(kpool2[used].view(torch.int16), kpool[used].view(torch.int16))
    assert kv2.free_pages() == kv.free_pages()


@pytest.mark.parametrize("D,ts,missing", [(64, 16, False), (128, 32, True), (128, 16, True),
                                           (32, 16, True), (256, 16, False), (256, 32, True)])
def test_grouped_attention_shared_prefix_random(gpu, oracle, D, ts, missing):
    """Beam-aware pa_decode_grouped on 3 sequences x 4 beams sharing a prefix
    of pages (the page table rows of a sequence's beams alias the same page
    ids), ragged per-row contexts, optionally missing pages (shared and
    private): equal to the oracle and to pa_decode."""
    import torch
    import llm_capi
    rng = np.random.default_rng(8 + D + ts)
    seqs, W, H, T = 3, 4, 4, 700
    B = seqs * W
    nt = (T + ts - 1) // ts
    shared = 30 * 16 // ts  # tiles shared by the beams of a sequence
    num_pages = seqs * H * shared + B * H * (nt - shared) + 3
    perm = rng.permutation(num_pages).astype(np.int32)
    pt = np.full((B, H, nt), -1, np.int32)
    i = 0
    for sq in range(seqs):
        blk = perm[i:i + H * shared].reshape(H, shared)
        i += H * shared
        for w in range(W):
            pt[sq * W + w, :, :shared] = blk
    for b in range(B):
        pt[b, :, shared:] = perm[i:i + H * (nt - shared)].reshape(H, nt - shared)
        i += H * (nt - shared)
    if missing:  # a shared tile (all 4 beams) and scattered private tiles
        pt[0:W, 1, 3] = -1
        pt[5, 2, shared + 1] = -1
        pt[9, 0, nt - 2] = -1
    kp = (rng.standard_normal((num_pages, ts, D)) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    d = lambda a: torch.from_numpy(a).cuda()
    # ragged contexts (groups fall back to per-wave loads), then equal contexts per
    # 4-beam group (the shared prefix pages go through the LDS prefetch)
    lens_ragged = rng.integers(shared * ts, T + 1, size=B).astype(np.int32)
    lens_equal = np.repeat(rng.integers(shared * ts, T + 1, size=seqs), W).astype(np.int32)
    for lens, bitwise in ((lens_ragged, True), (lens_equal, False)):
        ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T,
                                     context_lens=lens)
        plain = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T,
                                   context_lens=d(lens)).cpu().numpy()
        assert_parity(plain, ref, 1e-3)
        for g in (2, 4):
            outg = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                                      row_group=g).cpu().numpy()
            # ragged groups and groups of 2 keep the plain partition (bitwise);
            # equal-context groups of 4 split by cost (fp32 merge rounding only)
            if bitwise or g == 2:
                np.testing.assert_array_equal(outg, plain)
            else:
                assert rel_err(outg, plain) < 1e-5
            assert_parity(outg, ref, 1e-3)


@pytest.mark.parametrize("shared", [0, 1, 17, 43, 44])
@pytest.mark.parametrize("T", [700, 16 * 44 - 5])
@pytest.mark.parametrize("kvt", ["float16", "bfloat16"])
def test_grouped_attention_cost_balanced_splits(gpu, oracle, shared, T, kvt):
    """Beam groups whose 4 rows share the first `shared` of 44 tiles: the
    beam kernel splits the row by cost (a private tile is loaded per wave, a
    shared tile once per workgroup), and splits may be empty; every shared
    length from none to all, full and partial last tile, matches the oracle
    and the plain schedule to fp32 merge rounding."""
    import torch
    import llm_capi
    rng = np.random.default_rng(100 + shared + T)
    seqs, W, H, D, ts = 3, 4, 4, 128, 16
    B = seqs * W
    nt = 44
    num_pages = seqs * H * shared + B * H * (nt - shared) + 1
    perm = rng.permutation(num_pages).astype(np.int32)
    pt = np.full((B, H, nt), -1, np.int32)
    i = 0
    for sq in range(seqs):
        blk = perm[i:i + H * shared].reshape(H, shared)
        i += H * shared
        for w in range(W):
            pt[sq * W + w, :, :shared] = blk
    for b in range(B):
        pt[b, :, shared:] = perm[i:i + H * (nt - shared)].reshape(H, nt - shared)
        i += H * (nt - shared)
    kp = (rng.standard_normal((num_pages, ts, D)) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    d = lambda a: torch.from_numpy(a).cuda()
    # bf16 pools take the standard schedule (no beam kernel): bitwise the plain one
    kd = d(kp).to(getattr(torch, kvt))
    vd = d(vp).to(getattr(torch, kvt))
    kf, vf = kd.float().cpu().numpy(), vd.float().cpu().numpy()
    ref = oracle.paged_attention(q, kf, vf, pt, T=T)
    plain = llm_capi.pa_decode(d(q), kd, vd, d(pt), T=T).cpu().numpy()
    outg = llm_capi.pa_decode(d(q), kd, vd, d(pt), T=T, row_group=4).cpu().numpy()
    if kvt == "bfloat16":
        np.testing.assert_array_equal(outg, plain)
    assert_parity(plain, ref, 1e-3)
    assert_parity(outg, ref, 1e-3)
    assert rel_err(outg, plain) < 1e-5
    # fixed pages per split keep the uniform partition, empty splits included
    outf = llm_capi.pa_decode(d(q), kd, vd, d(pt), T=T, row_group=4,
                              pages_per_split=24).cpu().numpy()
    plainf = llm_capi.pa_decode(d(q), kd, vd, d(pt), T=T,
                                pages_per_split=24).cpu().numpy()
    np.testing.assert_array_equal(outf, plainf)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32", "int8"])
def test_typed_kv_cache_attention_and_save_load(gpu, oracle, tmp_path, dtype):
    """KVTileCache<T> for T in {bf16, float, int8_t} (kv_tile_cache.hpp:9):
    tokens written through the typed cache, attention through the pybind11
    paged_attention entry point, and a save/load round trip that keeps the
    element type (a cache of another type refuses the file)."""
    import torch
    import llm_decoder
    rng = np.random.default_rng(11)
    H, D, TS, T, B = 2, 64, 16, 70, 2
    dt = getattr(torch, dtype)
    kv = llm_decoder.KVTileCache()
    kv.init(num_pages=32, tile_size=TS, head_dim=D, num_layers=1, num_beams=B, num_heads=H,
            max_tiles=8, dtype=dtype)
    assert kv.view(0)["kv_dtype"] == {"bfloat16": 3, "float32": 2, "int8": 1}[dtype]
    ks, vs = [], []
    for b in range(B):
        if dtype == "int8":
            k = rng.integers(-4, 5, (T, H, D)).astype(np.int8)
            v = rng.integers(-4, 5, (T, H, D)).astype(np.int8)
            kf, vf = k.astype(np.float32), v.astype(np.float32)
        else:
            kt = torch.from_numpy(rng.standard_normal((T, H, D)).astype(np.float32) * 0.3).to(dt)
            vt = torch.from_numpy(rng.standard_normal((T, H, D)).astype(np.float32)).to(dt)
            kf, vf = kt.float().numpy(), vt.float().numpy()
            k = kt.view(torch.int16).numpy() if dtype == "bfloat16" else kt.numpy()
            v = vt.view(torch.int16).numpy() if dtype == "bfloat16" else vt.numpy()
        kv.write_tokens(0, b, 0, k, v)
        ks.append(kf)
        vs.append(vf)
    q = (rng.standard_normal((B, H, D)) * 0.1).astype(np.float32)
    qd = torch.from_numpy(q).cuda()
    out = torch.empty((B, H, D), device="cuda")
    ws_bytes = llm_decoder.workspace_bytes(B, H, D, 8)
    ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device="cuda")
    kv.sync_page_table_to_gpu()
    llm_decoder.paged_attention(kv.handle, 0, qd.data_ptr(), out.data_ptr(), B=B, H=H, D=D, T=T,
                                workspace=ws.data_ptr(), workspace_bytes=ws_bytes)
    torch.cuda.synchronize()
    # oracle over a dense per-(beam, head) pool built from what was written
    nt = (T + TS - 1) // TS
    kpool = np.zeros((B * H * nt, TS, D), np.float32)
    vpool = np.zeros_like(kpool)
    pt = np.arange(B * H * nt, dtype=np.int32).reshape(B, H, nt)
    for b in range(B):
        for h in range(H):
            for t in range(T):
                kpool[pt[b, h, t // TS], t % TS] = ks[b][t, h]
                vpool[pt[b, h, t // TS], t % TS] = vs[b][t, h]
    ref = oracle.paged_attention(q, kpool, vpool, pt, T=T)
    assert_parity(out.cpu().numpy(), ref, 1e-3)
    path = str(tmp_path / "kv.bin")
    kv.save_to_file(path, format="snapshot")
    kv2 = llm_decoder.KVTileCache()
    kv2.init(num_pages=32, tile_size=TS, head_dim=D, num_layers=1, num_beams=B, num_heads=H,
             max_tiles=8, dtype=dtype)
    kv2.load_from_file(path, format="snapshot")
    kv2.sync_page_table_to_gpu()
    out2 = torch.empty_like(out)
    llm_decoder.paged_attention(kv2.handle, 0, qd.data_ptr(), out2.data_ptr(), B=B, H=H, D=D,
                                T=T, workspace=ws.data_ptr(), workspace_bytes=ws_bytes)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    other = llm_decoder.KVTileCache()
    other.init(num_pages=32, tile_size=TS, head_dim=D, num_layers=1, num_beams=B, num_heads=H,
               max_tiles=8, dtype="float16")
    with pytest.raises(RuntimeError, match="kv_dtype"):
        other.load_from_file(path, format="snapshot")
