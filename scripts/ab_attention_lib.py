#!/usr/bin/env python3
"""Time the decode-attention launches of whichever library build LLM_CAPI_LIB
names (default: the in-tree one): the C3 plain launch (64 rows x 16 heads x
8192 tokens, shuffled interleaved pages) and a C4-shaped beam-group launch
(8 sequences x 4 beams, 3840 shared + 256 private tokens, row_group 4).
Run it once per build, alternating, to A/B compiler flags on one box.
    LLM_CAPI_LIB=path/to/lib.so python scripts/ab_attention_lib.py"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))


def timed(fn, iters=10):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import torch
    import llm_capi
    g = torch.Generator(device="cuda").manual_seed(0)
    H, D, ts = 16, 128, 16
    # C3 plain
    B, T = 64, 8192
    nt = T // ts
    n = B * H * nt
    kv = torch.randn((2 * n, ts, D), generator=g, device="cuda").half()
    pt = (2 * torch.randperm(n, generator=g, device="cuda")).to(torch.int32).reshape(B, H, nt)
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    c3 = timed(lambda: llm_capi.pa_decode(q, kv[:-1], kv[1:], pt, T=T))
    del kv
    # C4 shape: 8 seqs x 4 beams, 240 shared tiles + 16 private per beam
    S, W, T4 = 8, 4, 4096
    shared = int(os.environ.get("AB_C4_SHARED", 240))  # tiles of the forked prefix
    nt4 = T4 // ts
    B4 = S * W
    npages = S * H * shared + B4 * H * (nt4 - shared)
    kv4 = torch.randn((2 * npages, ts, D), generator=g, device="cuda").half()
    perm = 2 * torch.randperm(npages, generator=g, device="cuda").to(torch.int32)
    pt4 = torch.empty((B4, H, nt4), dtype=torch.int32, device="cuda")
    i = 0
    for s_ in range(S):
        blk = perm[i:i + H * shared].reshape(H, shared)
        i += H * shared
        for w in range(W):
            pt4[s_ * W + w, :, :shared] = blk
    for b in range(B4):
        pt4[b, :, shared:] = perm[i:i + H * (nt4 - shared)].reshape(H, nt4 - shared)
        i += H * (nt4 - shared)
    q4 = torch.randn((B4, H, D), generator=g, device="cuda") * D ** -0.25
    c4 = timed(lambda: llm_capi.pa_decode(q4, kv4[:-1], kv4[1:], pt4, T=T4, row_group=4))
    # the first C4 timing also pays first-touch costs; time the default again
    extra = {"c4_grouped_again_us": round(timed(lambda: llm_capi.pa_decode(
        q4, kv4[:-1], kv4[1:], pt4, T=T4, row_group=4)), 1)}
    for pps in [int(x) for x in os.environ.get("AB_C4_PPS", "").split(",") if x]:
        extra[f"c4_grouped_pps{pps}_us"] = round(timed(lambda: llm_capi.pa_decode(
            q4, kv4[:-1], kv4[1:], pt4, T=T4, row_group=4, pages_per_split=pps)), 1)
    print(json.dumps({"lib": os.environ.get("LLM_CAPI_LIB", "default"), "c3_us": round(c3, 1),
                      "c4_grouped_us": round(c4, 1)} | extra), flush=True)


if __name__ == "__main__":
    main()
