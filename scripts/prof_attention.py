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
        "c1": dict(B=1, H=4, D=64, T=128, ts=16),
        "c2": dict(B=16, H=12, D=64, T=2048, ts=16),
        "c5": dict(B=64, H=32, D=128, T=8192, ts=16),
        # C4: 8 sequences x 4 beams; each sequence's first 240 tiles are one
        # set of pages shared by its beams (kv_cache_fork), the last 16 private
        "c4": dict(B=32, H=16, D=128, T=4096, ts=16, beams=4, shared=240)}

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=sorted(CFGS))
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--decoder", action="store_true",
                help="time the decoder's own attention launch (llm_decoder_run_attention: the "
                     "step graph's kernels and outputs) of a 1-layer decoder of the config's dims")
args = ap.parse_args()
c = CFGS[args.config]
B, H, D, T, ts = c["B"], c["H"], c["D"], c["T"], c["ts"]
W = c.get("beams", 1)
if args.decoder:
    sys.path.insert(0, str(ROOT))
    import numpy as np  # noqa: E402
    import llm_decoder  # noqa: E402
    from bench import make_weights  # noqa: E402
    cls = "CUDADecoder" if args.config == "c2" else "INT8Decoder"
    cfg = dict(cls=cls, L=1, H=H, D=D, V=512)
    dec = getattr(llm_decoder, cls)(1, H, D, H * D, 512, T + 8, max_batch=B, page_size=ts)
    dec.set_weights(make_weights(cfg, 5))
    if W > 1:
        dec.begin_beams(B // W, W, c["shared"] * ts, T - c["shared"] * ts, 3, True)
    else:
        dec.begin_synthetic(B, T, 3, True)
    torch.cuda.set_stream(torch.cuda.Stream())
    st = torch.cuda.current_stream().cuda_stream
    dec.step(list(range(B)), stream=st)  # q rows of a real step; context T + 1
    T = dec.context_len(0)
    nt = (T + ts - 1) // ts
    nsplit, form = dec.attention_plan()

    def launch():
        dec.run_attention(0, st)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.iters):
        launch()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / args.iters * 1e-3
    kv_tiles = B * H * nt if W == 1 else (B // W) * H * (c["shared"] + W * (nt - c["shared"]))
    nbytes = 2 * kv_tiles * ts * D * 2 + B * H * nt * 4 + 2 * B * H * D * 4
    print(json.dumps({"config": args.config, "launch": "decoder (llm_decoder_run_attention)",
                      "nsplit": nsplit, "form": form, "T": T, "iters": args.iters,
                      "us_per_launch": round(t * 1e6, 2), "algorithmic_bytes": nbytes,
                      "GBps": round(nbytes / t / 1e9, 1)}))
    sys.exit(0)
nt = (T + ts - 1) // ts
num_pages = B * H * nt
g = torch.Generator(device="cuda").manual_seed(0)
# the kv_cache layout: K and V pages interleave ([num_pages][K page | V page])
kv = torch.randn((num_pages, 2, ts, D), generator=g, device="cuda").half()
kv[:, 0] *= D ** -0.25
kp, vp = kv[:, 0], kv[:, 1]
q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
pt = torch.randperm(num_pages, generator=g, device="cuda").to(torch.int32).reshape(B, H, nt)
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
