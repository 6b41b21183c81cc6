"""A/B the paged-attention split-kernel variants at the C3 shape in one process
(interleaved rounds, median), HIP-event timed.

    python scripts/tune_attention.py [--rounds 5] [--variants 0 1 2 3 4 5] [--pps 64]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import llm_capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--variants", type=int, nargs="*", default=[0, 1, 2, 3, 4, 5])
ap.add_argument("--pps", type=int, nargs="*", default=[64])
ap.add_argument("--T", type=int, default=8192)
ap.add_argument("--B", type=int, default=64)
ap.add_argument("--interleave", action="store_true",
                help="K and V of a page adjacent (one 2*page pool, K at even, V at odd pages)")
ap.add_argument("--extent", type=int, default=1,
                help="tiles per physically contiguous page run (1 = fully random pages; "
                     "nt = each (row, head) contiguous)")
ap.add_argument("--pool-pages", type=int, default=0,
                help="pages in each pool (>= B*H*tiles; the used pages are a random subset)")
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--v-gap", type=int, default=-1,
                help=">= 0: K and V pools in ONE allocation, V starting this many pages after K's end")
args = ap.parse_args()
B, H, D, T, ts = args.B, 16, 128, args.T, 16
nt = (T + ts - 1) // ts
num_pages = max(B * H * nt, args.pool_pages)
g = torch.Generator(device="cuda").manual_seed(args.seed)
if args.interleave:
    kv = torch.randn((2 * num_pages, ts, D), generator=g, device="cuda").half()
    kp, vp = kv[:-1], kv[1:]  # page p of kp = kv[p], of vp = kv[p + 1]
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    pt = (2 * torch.randperm(num_pages, generator=g, device="cuda")).to(torch.int32).reshape(B, H, nt)
else:
    kp = (torch.randn((num_pages, ts, D), generator=g, device="cuda") * D ** -0.25).half()
    vp = torch.randn((num_pages, ts, D), generator=g, device="cuda").half()
    if args.v_gap >= 0:
        both = torch.empty((2 * num_pages + args.v_gap, ts, D), device="cuda", dtype=torch.half)
        both[:num_pages] = kp
        both[num_pages + args.v_gap:] = vp
        del kp, vp
        kp, vp = both[:num_pages], both[num_pages + args.v_gap:]
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    pt = torch.randperm(num_pages, generator=g, device="cuda").to(torch.int32)[:B * H * nt].reshape(B, H, nt)
if args.extent > 1 and not args.interleave:
    ext = args.extent
    assert nt % ext == 0
    runs = torch.randperm(num_pages // ext, generator=g, device="cuda").to(torch.int32)
    pt = (runs[:, None] * ext + torch.arange(ext, device="cuda", dtype=torch.int32)).reshape(B, H, nt)
lib = llm_capi.load_tune()  # tuning build: `make tune`
lib.pa_decode_tune.restype = ctypes.c_int
lib.pa_decode_tune.argtypes = [ctypes.c_int, ctypes.POINTER(llm_capi.PaKvView), ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_void_p]
view = llm_capi.kv_view(kp, vp, pt)
out = torch.empty((B, H, D), device="cuda")
ref = llm_capi.pa_decode(q, kp, vp, pt, T=T)
ws_bytes = lib.pa_decode_workspace_bytes(B, H, D, nt, 1)
ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda")
st = llm_capi.stream_ptr()
nbytes = 2 * B * H * T * D * 2 + B * H * nt * 4
res = {}
for r in range(args.rounds):
    for pps in args.pps:
        for v in args.variants:
            def run():
                llm_capi.check(lib.pa_decode_tune(v, ctypes.byref(view), llm_capi.ptr(q),
                                                  llm_capi.ptr(out), None, B, H, T, pps,
                                                  llm_capi.ptr(ws), ws_bytes, st))
            run()
            torch.cuda.synchronize()
            if r == 0 and (v < 10 or 13 <= v < 19 or v >= 20) and v not in (24, 25):  # load-only ceilings: 10-12, 19, 24, 25
                err = (out - ref).abs().max().item() / ref.abs().max().item()
                assert err < 1e-5, (v, pps, err)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                run()
            e.record()
            torch.cuda.synchronize()
            res.setdefault((v, pps), []).append(s.elapsed_time(e) / args.iters * 1e-3)
for (v, pps), ts_ in sorted(res.items()):
    t = float(np.median(ts_))
    print(json.dumps({"variant": v, "pps": pps, "us": round(t * 1e6, 1),
                      "GBps": round(nbytes / t / 1e9, 1), "frac_8TBps": round(nbytes / t / 8e12, 4),
                      "min_us": round(min(ts_) * 1e6, 1)}))
