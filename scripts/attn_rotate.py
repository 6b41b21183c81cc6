"""The decoder's attention launch timed two ways (HIP events, torch's stream):
layer 0 relaunched back to back (bench.py's time_attention) and the launches
rotating over every layer (each launch reads another layer's KV zone, as the
step does).  A KV working set that fits the 256 MiB Infinity Cache (C2: 101 MB
per layer) is re-served from it in the first form only.

    python scripts/attn_rotate.py [--config c2] [--iters 48]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--iters", type=int, default=48)
    a = ap.parse_args()
    import torch
    import bench
    import llm_decoder
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    cfg = bench.CONFIGS[a.config]
    dec = getattr(llm_decoder, cfg["cls"])(cfg["L"], cfg["H"], cfg["D"], cfg["H"] * cfg["D"],
                                           cfg["V"], cfg["T"] + 16, max_batch=cfg["B"],
                                           page_size=cfg["ts"])
    dec.set_weights(bench.make_weights(cfg, 1234))
    dec.begin_synthetic(cfg["B"], cfg["T"], 1234, True)
    st = torch.cuda.current_stream().cuda_stream
    dec.step(list(range(cfg["B"])), stream=st)
    torch.cuda.synchronize()

    def timed(layers):
        for l in layers[:3]:
            dec.run_attention(l, st)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for l in layers:
            dec.run_attention(l, st)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / len(layers) * 1e3
    same = timed([0] * a.iters)
    rot = timed([i % cfg["L"] for i in range(a.iters)])
    same2 = timed([0] * a.iters)
    print(f"{a.config}: layer 0 back to back {same:.2f} / {same2:.2f} us, rotating over "
          f"{cfg['L']} layers {rot:.2f} us per launch")


if __name__ == "__main__":
    main()
