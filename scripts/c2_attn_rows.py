"""C2 attention launch time against the row count (FP16 decoder, H 12, D 64,
T 2048): does the workgroup-merge launch (one workgroup per (row, head))
scale with the CUs it occupies?  16 rows = 192 workgroups on 256 CUs.

    python scripts/c2_attn_rows.py [--rows 16 21 32 48]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import llm_decoder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, nargs="*", default=[16, 21, 24, 32, 48])
ap.add_argument("--T", type=int, default=2048)
ap.add_argument("--layers", type=int, default=1)
args = ap.parse_args()
cfg = dict(bench.CONFIGS["c2"], L=args.layers)
hid = cfg["H"] * cfg["D"]
w = bench.make_weights(cfg, 0)
torch.cuda.set_stream(torch.cuda.Stream())  # handle 0 would be the decoder's own stream
for B in args.rows:
    dec = llm_decoder.CUDADecoder(cfg["L"], cfg["H"], cfg["D"], hid, cfg["V"], args.T + 16,
                                  max_batch=B, page_size=cfg["ts"])
    dec.set_weights(w)
    dec.begin_synthetic(B, args.T, 1, True)
    logits = torch.empty((B, cfg["V"]), device="cuda")
    for _ in range(2):  # the step uploads the rows' contexts
        dec.step([1] * B, logits_ptr=logits.data_ptr(),
                 stream=torch.cuda.current_stream().cuda_stream, want_next=False)
    torch.cuda.synchronize()
    ns, form = dec.attention_plan()
    ts = sorted(bench.time_attention(dec, 1, iters=50) for _ in range(5))
    t = ts[2]
    by = bench.attention_launch_bytes(cfg, dec.context_len(0), B)
    print(f"ctx {dec.context_len(0)} ", end="")
    print(f"rows {B:3d} wgs {B * cfg['H']:4d} splits {ns} form {form:#x}: {t * 1e6:7.2f} us "
          f"{by / t / 1e12:5.2f} TB/s  {t * 1e6 / B:6.3f} us/row", flush=True)
    del dec
    torch.cuda.synchronize()
