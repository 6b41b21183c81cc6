"""Run the production paged-attention launch (split + merge) at a BASELINE
config shape a fixed number of times, for rocprofv3 kernel-trace / PMC passes:

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o att -- \
        python3 scripts/prof_attention.py --config c3 --iters 20
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o fetch -- \
        python3 scripts/prof_attention.py --config c3 --iters 20

KV pools hold seeded random fp16 and pages are a shuffled permutation of the
pool, so the gather is non-contiguous; K and V pages interleave
as in the decoder's kv_cache.
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))

import torch  # noqa: E402

import llm_capi  # noqa: E402

CFGS = {"c3": dict(B=64, H=16, D=128, T=8192, ts=16),
        "c2": dict(B=16, H=12, D=64, T=2048, ts=16),
        # C4: 8 sequences x 4 beams; each sequence's first 240 tiles are one
        # set of pages shared by its beams (kv_cache_fork), the last 16 private
        "c4": dict(B=32, H=16, D=128, T=4096, ts=16, beams=4, shared=240)}

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=sorted(CFGS))
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
c = CFGS[args.config]
B, H, D, T, ts = c["B"], c["H"], c["D"], c["T"], c["ts"]
nt = (T + ts - 1) // ts
num_pages = B * H * nt
g = torch.Generator(device="cuda").manual_seed(0)
# the kv_cache layout: K and V pages interleave ([num_pages][K page | V page])
kv = torch.randn((num_pages, 2, ts, D), generator=g, device="cuda").half()
kv[:, 0] *= D ** -0.25
kp, vp = kv[:, 0], kv[:, 1]
q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
pt = torch.randperm(num_pages, generator=g, device="cuda").to(torch.int32).reshape(B, H, nt)
W = c.get("beams", 1)
if W > 1:  # beams of a sequence alias the first `shared` page ids of its first beam
    sh = c["shared"]
    pt = pt.reshape(B // W, W, H, nt).clone()
    pt[:, 1:, :, :sh] = pt[:, :1, :, :sh]
    pt = pt.reshape(B, H, nt).contiguous()
out = torch.empty((B, H, D), device="cuda")
lib = llm_capi.load()
view = llm_capi.kv_view(kp, vp, pt)
pps = 0  # production choice: balanced device-side splits
ws_bytes = lib.pa_decode_workspace_bytes(B, H, D, nt, 0)
ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device="cuda")
st = llm_capi.stream_ptr()


def launch():
    if W > 1:
        llm_capi.check(lib.pa_decode_grouped(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out),
                                             None, None, B, H, D, T, 1.0, pps, W,
                                             llm_capi.ptr(ws), ws_bytes, st))
    else:
        llm_capi.check(lib.pa_decode(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out), None,
                                     None, B, H, D, T, 1.0, pps, llm_capi.ptr(ws), ws_bytes, st))


for _ in range(3):  # warm-up (first-touch / TLB)
    launch()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(args.iters):
    launch()
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / args.iters * 1e-3
# unique K/V bytes (a shared page counts once per sequence) + page table + q/out
kv_tiles = B * H * nt if W == 1 else (B // W) * H * (c["shared"] + W * (nt - c["shared"]))
nbytes = 2 * kv_tiles * ts * D * 2 + B * H * nt * 4 + 2 * B * H * D * 4
print(json.dumps({"config": args.config, "pps": pps, "iters": args.iters,
                  "us_per_launch": round(t * 1e6, 2), "algorithmic_bytes": nbytes,
                  "GBps": round(nbytes / t / 1e9, 1)}))
