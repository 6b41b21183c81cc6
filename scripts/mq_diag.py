"""Diagnostic for the tuning build's pa_beam_mq_kernel (LLM_BEAM4=2): small
cases against the one-wave-per-group kernel (LLM_BEAM4=1), per-(row, head)
relative error and a few output values.  GPU box only; prints to stdout."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "pagedattention-based-transformer-decoder-inference-framework_amd"))
import llm_capi  # noqa: E402


def case(B, H, T, shared, seed=0):
    rng = np.random.default_rng(seed)
    D, ts = 128, 16
    nt = (T + ts - 1) // ts
    npg = H * nt * B + 2
    pt = np.arange(B * H * nt, dtype=np.int32).reshape(B, H, nt)
    if shared:
        pt[:, :, :shared] = pt[0:1, :, :shared]
    kp = (rng.standard_normal((npg, ts, D)) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((npg, ts, D)).astype(np.float16)
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    lens = np.full(B, T, np.int32)
    d = lambda a: torch.from_numpy(a).cuda()
    outs = {}
    for mode in ("1", "2"):
        os.environ["LLM_BEAM4"] = mode
        outs[mode] = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                                        row_group=4, lib=llm_capi.load_tune()).cpu().numpy()
    a, b = outs["1"].reshape(B, H, D), outs["2"].reshape(B, H, D)
    print(f"B={B} H={H} T={T} shared={shared}")
    for r in range(B):
        for h in range(H):
            e = np.abs(a[r, h] - b[r, h]).max() / max(np.abs(a[r, h]).max(), 1e-30)
            print(f"  row {r} head {h}: rel {e:.3e}  ref[:4] {a[r, h, :4]}  mq[:4] {b[r, h, :4]}"
                  f"  ratio(med) {np.median(b[r, h] / a[r, h]):.4f}")
    sys.stdout.flush()


if __name__ == "__main__":
    case(4, 1, 16, 1)
    case(4, 1, 16, 0)
    case(1, 1, 16, 0)
    case(4, 1, 64, 4)
    case(4, 2, 700, 30)
