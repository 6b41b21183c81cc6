#!/usr/bin/env python3
"""Prefill attention: the MFMA chunk kernel (pa_prefill) against the same rows
through the decode kernel (pa_decode with beam_ids = row, context_lens =
p0 + i + 1), and a whole-decoder prompt prefill (MFMA prefill kernel).

    python scripts/bench_prefill.py [--p0 7680] [--m 512] [--prompt 4096]

Prints one JSON line.  Attention flops are algorithmic (4·H·D per (query,
key) pair, causal pairs only), not the hi/lo MFMA count."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
sys.path.insert(0, str(ROOT))


def time_cuda(fn, iters=10):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def kernel_bench(H, D, ts, p0, m):
    import torch
    import llm_capi
    rng = np.random.default_rng(0)
    T = p0 + m
    nt = (T + ts - 1) // ts
    num_pages = H * nt + 3
    kp = torch.from_numpy((rng.standard_normal((num_pages, ts, D)) * D ** -0.25).astype(np.float16)).cuda()
    vp = torch.from_numpy(rng.standard_normal((num_pages, ts, D)).astype(np.float16)).cuda()
    pt = torch.from_numpy(rng.permutation(num_pages)[:H * nt].astype(np.int32).reshape(1, H, nt)).cuda()
    q = torch.from_numpy((rng.standard_normal((m, H, D)) * D ** -0.25).astype(np.float32)).cuda()
    out = torch.empty((m, H, D), dtype=torch.float32, device="cuda")
    bi = torch.zeros(m, dtype=torch.int32, device="cuda")
    cl = torch.arange(p0 + 1, T + 1, dtype=torch.int32, device="cuda")
    t_pf = time_cuda(lambda: llm_capi.pa_prefill(q, kp, vp, pt, row=0, p0=p0, out=out))
    t_dec = time_cuda(lambda: llm_capi.pa_decode(q, kp, vp, pt, T=T, beam_ids=bi, context_lens=cl))
    pairs = m * p0 + m * (m + 1) // 2
    flops = 4.0 * H * D * pairs
    return {"H": H, "D": D, "page": ts, "p0": p0, "m": m, "prefill_us": round(t_pf, 1),
            "decode_rows_us": round(t_dec, 1), "speedup": round(t_dec / t_pf, 2),
            "prefill_TFLOPs": round(flops / t_pf / 1e6, 1),
            "kv_unique_GB": round(2 * H * T * D * 2 / 1e9, 4)}


def decoder_bench(prompt):
    import llm_decoder
    from bench import CONFIGS, make_weights
    cfg = CONFIGS["c3"]
    hid = cfg["H"] * cfg["D"]
    dec = llm_decoder.INT8Decoder(cfg["L"], cfg["H"], cfg["D"], hid, cfg["V"], prompt + 64,
                                  max_batch=1, page_size=cfg["ts"])
    dec.set_weights(make_weights(cfg, 1234))
    toks = np.random.default_rng(1).integers(0, cfg["V"], prompt).tolist()
    dec.begin_synthetic(1, 0, 1, True)
    dec.prefill(0, toks[:512])  # warm
    dec.sync()
    dec.begin_synthetic(1, 0, 1, True)
    t0 = time.perf_counter()
    dec.prefill(0, toks)
    dec.sync()
    dt = time.perf_counter() - t0
    del dec
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p0", type=int, default=7680)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=4096)
    ap.add_argument("--no-decoder", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    res = {"kernel": [kernel_bench(16, 128, 16, args.p0, args.m),
                      kernel_bench(16, 128, 16, 0, args.m),
                      kernel_bench(12, 64, 16, 1536, args.m)]}
    if not args.no_decoder:
        t1 = decoder_bench(args.prompt)
        res["decoder"] = {"config": "C3 dims (24L/16H/D128, INT8), batch 1",
                          "prompt_tokens": args.prompt, "mfma_prefill_s": round(t1, 3),
                          "mfma_prompt_tok_per_s": round(args.prompt / t1, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
