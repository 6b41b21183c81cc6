"""Run the C-ABI LM head (pack + lm_head_kernel) at the C3 shape a fixed number
of times, for rocprofv3 kernel-trace timing of lm_head_kernel; prints the max
abs difference against a torch fp32 reference of x . E^T.
    rocprofv3 --kernel-trace --stats -d OUT -- python3 scripts/time_lm_head.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

import os  # noqa: E402
M, V, K = (int(v) for v in os.environ.get("LM_SHAPE", "64,50257,2048").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn((M, K), generator=g, device="cuda")
E = (torch.randn((V, K), generator=g, device="cuda") * 0.02).half()
for _ in range(20):
    out = llm_capi.lm_head(x, E)
torch.cuda.synchronize()
ref = x @ E.float().t()
print("max_abs_err", (out - ref).abs().max().item(), "ref_max", ref.abs().max().item())
