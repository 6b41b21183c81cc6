"""Time pa_decode (split + merge, HIP events) at one config shape over a list
of pages_per_split values (0 = the production choice); interleaved K/V pages
as in the decoder's kv_cache.

    python scripts/sweep_attention_pps.py --B 16 --H 12 --D 64 --T 2048 --pps 0 4 8 16 32
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=16)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--D", type=int, default=64)
ap.add_argument("--T", type=int, default=2048)
ap.add_argument("--ts", type=int, default=16)
ap.add_argument("--pps", type=int, nargs="*", default=[0, 4, 8, 16, 32])
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
nt = (a.T + a.ts - 1) // a.ts
n = a.B * a.H * nt
g = torch.Generator(device="cuda").manual_seed(0)
kv = torch.randn((2 * n, a.ts, a.D), generator=g, device="cuda").half()
pt = (2 * torch.randperm(n, generator=g, device="cuda")).to(torch.int32).reshape(a.B, a.H, nt)
q = torch.randn((a.B, a.H, a.D), generator=g, device="cuda") * a.D ** -0.25
nbytes = 2 * a.B * a.H * a.T * a.D * 2 + a.B * a.H * nt * 4 + 2 * a.B * a.H * a.D * 4
import ctypes  # noqa: E402
lib = llm_capi.load()
view = llm_capi.kv_view(kv[:-1], kv[1:], pt)
out = torch.empty((a.B, a.H, a.D), device="cuda")
ws_bytes = max(lib.pa_decode_workspace_bytes(a.B, a.H, a.D, nt, 1),
               lib.pa_decode_workspace_bytes(a.B, a.H, a.D, nt, 0))
ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda")
st = llm_capi.stream_ptr()
ref = llm_capi.pa_decode(q, kv[:-1], kv[1:], pt, T=a.T)
res = {}
for _ in range(a.rounds):
    for pps in a.pps:
        def fn(pps=pps):  # raw C-ABI launch, buffers preallocated (GPU-bound timing)
            llm_capi.check(lib.pa_decode(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out),
                                         None, None, a.B, a.H, a.D, a.T, 1.0, pps,
                                         llm_capi.ptr(ws), ws_bytes, st))
        fn()
        torch.cuda.synchronize()
        assert (out - ref).abs().max().item() <= 1e-4 * ref.abs().max().item(), pps
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.setdefault(pps, []).append(s.elapsed_time(e) / a.iters * 1e3)
for pps, v in res.items():
    t = min(v)
    print(json.dumps({"pps": pps, "us": round(t, 2), "TBps": round(nbytes / t / 1e6, 2)}))
