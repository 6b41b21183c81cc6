"""Kernel-level timing of the decode hot path on one MI355X (HIP events).

    python scripts/bench_kernels.py [--config c3|c2] [--iters N]

Prints one line per kernel: avg time, algorithmic bytes, GB/s, % of 8 TB/s.
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))

import torch  # noqa: E402

import llm_capi  # noqa: E402

PEAK = 8.0e12


def timeit(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pps", type=int, nargs="*", default=[0])
    args = ap.parse_args()
    cfg = {"c3": dict(B=64, H=16, D=128, T=8192, ts=16, V=50257),
           "c2": dict(B=16, H=12, D=64, T=2048, ts=16, V=50257)}[args.config]
    B, H, D, T, ts, V = (cfg[k] for k in ("B", "H", "D", "T", "ts", "V"))
    hid = H * D
    nt = (T + ts - 1) // ts
    num_pages = B * H * nt
    g = torch.Generator(device="cuda").manual_seed(0)
    kp = (torch.randn((num_pages, ts, D), generator=g, device="cuda") * D ** -0.25).half()
    vp = torch.randn((num_pages, ts, D), generator=g, device="cuda").half()
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    pt = torch.randperm(num_pages, generator=g, device="cuda").to(torch.int32).reshape(B, H, nt)
    res = []
    attn_bytes = 2 * B * H * T * D * 2 + B * H * nt * 4 + 2 * B * hid * 4
    for pps in args.pps:
        out = torch.empty((B, H, D), device="cuda")
        view = llm_capi.kv_view(kp, vp, pt)
        lib = llm_capi.load()
        ws_bytes = lib.pa_decode_workspace_bytes(B, H, D, nt, pps)
        ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device="cuda")
        import ctypes
        st = llm_capi.stream_ptr()

        def run():
            llm_capi.check(lib.pa_decode(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out),
                                         None, None, B, H, D, T, 1.0, pps, llm_capi.ptr(ws),
                                         ws_bytes, st))
        t = timeit(run, args.iters)
        res.append(dict(kernel=f"pa_decode(pps={pps or lib.pa_decode_pages_per_split(B, H, T, ts, nt)})",
                        us=t * 1e6, bytes=attn_bytes, GBps=attn_bytes / t / 1e9,
                        frac=attn_bytes / t / PEAK))
    del kp, vp
    torch.cuda.empty_cache()
    M = B
    for name, K, N in [("qkv_proj", hid, 3 * hid), ("o_proj", hid, hid), ("mlp_fc1", hid, 4 * hid),
                       ("mlp_fc2", 4 * hid, hid)]:
        W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
        Wp = llm_capi.pack_weights(W, llm_capi.LLM_I8)
        A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda")
        sa = torch.rand(M, device="cuda")
        sw = torch.rand(N, device="cuda")
        t = timeit(lambda: llm_capi.i8_gemm(A, Wp, N, sa=sa, sw=sw, want_acc=False), args.iters)
        byts = K * N + M * K + M * N * 4 + 4 * (M + N)
        res.append(dict(kernel=f"i8_gemm {name} M{M} K{K} N{N}", us=t * 1e6, bytes=byts,
                        GBps=byts / t / 1e9, frac=byts / t / PEAK,
                        TOPS=2 * M * K * N / t / 1e12))
    E = torch.randn((V, hid), device="cuda").half()
    x = torch.randn((M, hid), device="cuda")
    t = timeit(lambda: llm_capi.lm_head(x, E), args.iters)
    byts = V * hid * 2 + M * hid * 4 + M * V * 4
    res.append(dict(kernel=f"lm_head M{M} V{V} K{hid}", us=t * 1e6, bytes=byts,
                    GBps=byts / t / 1e9, frac=byts / t / PEAK))
    logits = torch.randn((M, V), device="cuda")
    t = timeit(lambda: llm_capi.argmax_rows(logits), args.iters)
    res.append(dict(kernel="argmax", us=t * 1e6))
    for r in res:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
