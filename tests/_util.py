"""Shared test helpers: golden fixture loading and page-pool construction."""
from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"
RECORD_DIR = Path(os.environ.get("LLM_RECORD_DIR",
                                 Path(__file__).resolve().parents[1] / "gpurun_out"))


def record(name: str, **kv) -> None:
    """Append one JSON line of measured figures to RECORD_DIR/<name>.jsonl (the
    GPU box's gpurun_out/, copied into profiles/ for the record)."""
    RECORD_DIR.mkdir(parents=True, exist_ok=True)
    with open(RECORD_DIR / f"{name}.jsonl", "a") as f:
        f.write(json.dumps(kv) + "\n")


def load_attn_fixture(name: str) -> dict:
    z = np.load(GOLDEN / f"attn_{name}.npz")
    B, H, D, T, ts, beams, top_k, eos = (int(x) for x in z["params"])
    temperature, top_p, eos_thr = (float(x) for x in z["fparams"])
    return dict(q=z["q"], k=z["k"], v=z["v"], present=z["present"],
                beam_ids=z["beam_ids"] if z["beam_ids"].size else None,
                B=B, H=H, D=D, T=T, ts=ts, beams=beams, top_k=top_k, eos=eos,
                temperature=temperature, top_p=top_p, eos_thr=eos_thr,
                out=z["out"], probs=z["probs"], scores=z["scores"])


def tiles_to_pool(k_tiles, v_tiles, present, *, seed=7, extra_pages=3):
    """Scatter per-(beam, head, tile) tiles into a shuffled page pool.

    Returns (k_pool, v_pool, page_table) with pools [num_pages][ts][D] (same
    dtype as the tiles) and page_table int32 [beams][H][ntiles] (-1 where the
    tile is absent).  Unused pool pages are filled with garbage so a wrong
    page lookup cannot pass by accident."""
    beams, H, nt, ts, D = k_tiles.shape
    n = beams * H * nt
    num_pages = n + extra_pages
    rng = np.random.default_rng(seed)
    perm = rng.permutation(num_pages)[:n]
    k_pool = (rng.standard_normal((num_pages, ts, D)) * 50).astype(k_tiles.dtype)
    v_pool = (rng.standard_normal((num_pages, ts, D)) * 50).astype(v_tiles.dtype)
    pt = np.full((beams, H, nt), -1, np.int32)
    i = 0
    for r in range(beams):
        for h in range(H):
            for t in range(nt):
                if present[r, h, t]:
                    pt[r, h, t] = perm[i]
                    k_pool[perm[i]] = k_tiles[r, h, t]
                    v_pool[perm[i]] = v_tiles[r, h, t]
                i += 1
    return k_pool, v_pool, pt


def rel_err(a, b):
    """Tensor-normalised error max|a - b| / max|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def elem_err(a, b, rtol=1e-3, atol_frac=1e-6, axis=None):
    """Worst elementwise ratio |a - b| / (rtol |b| + atol_frac max|b|) (<= 1
    passes): every element within rtol of its own value, with an absolute
    floor of atol_frac of the largest |b| (of the whole tensor, or of each
    slice along `axis`, e.g. per logit row)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.max(np.abs(b), axis=axis, keepdims=axis is not None) if b.size else 0.0
    tol = rtol * np.abs(b) + atol_frac * np.maximum(scale, 1e-30)
    return float(np.max(np.abs(a - b) / tol)) if b.size else 0.0


def assert_parity(a, b, rtol=1e-3, atol_frac=1e-6, axis=None, what=""):
    """The north_star's "1e-3 rel" as both bounds: tensor-normalised
    (rel_err < rtol) and elementwise (|a - b| <= rtol |b| + atol_frac max|b|,
    SURVEY Appendix B.1)."""
    r = rel_err(a, b)
    e = elem_err(a, b, rtol, atol_frac, axis)
    assert r < rtol, f"{what} rel_err {r:.3e} >= {rtol}"
    if e > 1.0:
        a64, b64 = np.asarray(a, np.float64), np.asarray(b, np.float64)
        i = np.unravel_index(np.argmax(np.abs(a64 - b64) / (rtol * np.abs(b64) + 1e-300)), b64.shape)
        raise AssertionError(f"{what} elementwise bound exceeded x{e:.2f} "
                             f"(worst rel element {i}: {a64[i]!r} vs {b64[i]!r}; rel_err {r:.3e})")


def hip_copy_to_host(dst: np.ndarray, src_ptr: int) -> None:
    """hipMemcpy device -> host of dst.nbytes bytes (tests that read the
    decoder's pools and page tables back)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipMemcpy.restype = ctypes.c_int
    assert hip.hipMemcpy(dst.ctypes.data, ctypes.c_void_p(src_ptr), dst.nbytes, 2) == 0


def decoder_kv_to_oracle(dec, odec, rows, T):
    """Copy the decoder's paged KV context (positions [0, T) of every row, every
    layer, read back from its page pools through its page table) into the
    oracle decoder's contiguous KV (OracleDecoder.kv).  Returns the number of
    distinct pages read per layer (beam forks share pages)."""
    import ctypes
    import llm_capi
    lib = llm_capi.load()
    kvh = ctypes.c_void_p(dec.kv_handle)
    view = llm_capi.PaKvView()
    llm_capi.check(lib.kv_cache_view(kvh, 0, ctypes.byref(view)))
    ts, D, H, mt = view.page_size, view.head_dim, view.num_heads, view.max_tiles
    n_pages = lib.kv_cache_num_pages(kvh)
    stride = lib.kv_cache_page_stride(kvh)  # bytes from page to page (K page | V page)
    assert stride == 2 * ts * D * 2, stride
    pool = np.empty((n_pages, 2, ts, D), np.float16)
    hip_copy_to_host(pool, lib.kv_cache_k_pool(kvh))
    nt = (T + ts - 1) // ts
    c = odec.cfg
    distinct = []
    for layer in range(c["L"]):
        pt = np.empty((view.num_beams, H, mt), np.int32)
        hip_copy_to_host(pt, lib.kv_cache_page_table(kvh, layer))
        ids = pt[:rows, :, :nt]
        assert (ids >= 0).all() and (ids < n_pages).all()
        distinct.append(len(np.unique(ids)))
        for which in (0, 1):
            kv = odec.kv(layer, which)  # [B][H][max_seq][D]
            pages = pool[ids, which]    # [rows][H][nt][ts][D]
            kv[:rows, :, :T] = pages.reshape(rows, H, nt * ts, D)[:, :, :T]
    return distinct


def decoder_kv_at(dec, rows, pos, L):
    """The K and V the decoder's last step appended: fp16 [L][rows][2][H][D] at
    position pos[r] of each row, read back from its pages (teacher forcing of
    the fp16 decoder's KV append: OracleDecoder.step_attn(forced_kv=...))."""
    import ctypes
    import llm_capi
    lib = llm_capi.load()
    kvh = ctypes.c_void_p(dec.kv_handle)
    view = llm_capi.PaKvView()
    llm_capi.check(lib.kv_cache_view(kvh, 0, ctypes.byref(view)))
    ts, D, H, mt = view.page_size, view.head_dim, view.num_heads, view.max_tiles
    stride = lib.kv_cache_page_stride(kvh)
    base = lib.kv_cache_k_pool(kvh)
    out = np.empty((L, rows, 2, H, D), np.float16)
    page = np.empty((2, ts, D), np.float16)
    for layer in range(L):
        pt = np.empty((view.num_beams, H, mt), np.int32)
        hip_copy_to_host(pt, lib.kv_cache_page_table(kvh, layer))
        for r in range(rows):
            p = int(pos[r])
            for h in range(H):
                pg = int(pt[r, h, p // ts])
                assert pg >= 0
                hip_copy_to_host(page, base + pg * stride)
                out[layer, r, :, h] = page[:, p % ts]
    return out
