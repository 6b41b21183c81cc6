"""One page, 4 beams sharing it, V = one-hot rows: the output row of each beam
is its softmax weight vector over the 16 tokens (MFMA beam kernel vs numpy)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import llm_capi  # noqa: E402

np.set_printoptions(precision=4, suppress=True, linewidth=200)
for npg, pps in ((4, 1), (4, 2), (8, 4), (16, 4), (16, 8), (16, 0), (32, 4), (32, 16)):
    rng = np.random.default_rng(1)
    B, H, D, ts = 4, 1, 128, 16
    T = ts * npg
    pt = np.arange(npg, dtype=np.int32).reshape(1, 1, npg).repeat(B, 0)
    kp = (rng.standard_normal((npg, ts, D)) * 0.3).astype(np.float16)
    vp = np.zeros((npg, ts, D), np.float16)
    for t in range(T):
        vp[t // ts, t % ts, t % D] = 1.0
    q = rng.standard_normal((B, H, D)).astype(np.float32) * 0.3
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    o = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, row_group=4, pages_per_split=pps).cpu().numpy()
    K = kp.reshape(T, D).astype(np.float64)
    V = vp.reshape(T, D).astype(np.float64)
    s = np.einsum("bhd,td->bht", q.astype(np.float64), K)
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    want = np.einsum("bht,td->bhd", p, V)
    print(npg, "pages pps", pps, ": max err", np.abs(o - want).max(), "sum gpu", o[:, 0].sum(-1), flush=True)
