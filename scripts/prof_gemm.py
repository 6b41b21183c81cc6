#!/usr/bin/env python3
"""Driver for GEMM counters: a bench config's decoder (PROF_CONFIG: c3 INT8 24 L /
16 H / D 128, 64 rows; c5 INT8 32 H / D 128, 64 rows; c2 FP16 12 H / D 64, 16
rows) stepped eagerly (LLM_GRAPH=0, so every kernel is its own dispatch) at a
short context -- the weight GEMMs are the same launches as in the 8192-token
bench (their shapes do not depend on the context).  PROF_LAYERS (default: the
config's) limits the layer count, which changes only how many dispatches of
each GEMM are sampled.  Used under rocprofv3 by scripts/gpu_gemm_pmc.sh."""
import os
import sys
from pathlib import Path

os.environ.setdefault("LLM_GRAPH", "0")
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import llm_decoder
    from bench import CONFIGS, make_weights
    torch.cuda.set_device(0)
    cfg = dict(CONFIGS[os.environ.get("PROF_CONFIG", "c3")])
    cfg["L"] = int(os.environ.get("PROF_LAYERS", cfg["L"]))
    hid = cfg["H"] * cfg["D"]
    dec = getattr(llm_decoder, cfg["cls"])(cfg["L"], cfg["H"], cfg["D"], hid, cfg["V"], 512,
                                           max_batch=cfg["B"], page_size=cfg["ts"])
    dec.set_weights(make_weights(cfg, 1234))
    dec.begin_synthetic(cfg["B"], 256, 1, True)
    for i in range(int(os.environ.get("PROF_STEPS", "3"))):
        dec.step(list(range(cfg["B"])) if i == 0 else None, want_next=False)
    dec.sync()


if __name__ == "__main__":
    main()
