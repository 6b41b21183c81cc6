"""Shared test helpers: golden fixture loading and page-pool construction."""
from __future__ import annotations

from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


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
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))
