#!/usr/bin/env python3
"""C2 seam experiment: the FP16 decoder's o_proj -> LN2 + fc1 (16 rows, hid
768, inter 3072) as the decoder's two launches vs ONE launch with an in-kernel
device-scope arrival counter (f16_gemm_pair_tune, tuning build).  Checks the
two give bit-identical outputs, then times each graph-replayed (REPS pairs per
replay, best of 5 replays).
    python scripts/seam_pair.py [--reps 100]"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=100)
ap.add_argument("--M", type=int, default=16)
ap.add_argument("--hid", type=int, default=768)
ap.add_argument("--inter", type=int, default=3072)
args = ap.parse_args()
lib = llm_capi.load_tune()
f = lib.f16_gemm_pair_tune
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
M, K, N2 = args.M, args.hid, args.inter
torch.manual_seed(0)
dev = "cuda"
A = (torch.randn(M, K, device=dev) * 0.5).half()
Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_F16)  # A-fragment order
W1 = llm_capi.pack_weights((torch.randn(K, K, device=dev) * 0.03).half(), llm_capi.LLM_F16)
W2 = llm_capi.pack_weights((torch.randn(K, N2, device=dev) * 0.03).half(), llm_capi.LLM_F16)
g = torch.rand(K, device=dev) + 0.5
b = torch.randn(K, device=dev) * 0.1
b2 = torch.randn(N2, device=dev) * 0.1
sync = torch.zeros(4, dtype=torch.int32, device=dev)
outs = {}
s = torch.cuda.Stream()
res = {"M": M, "hid": K, "inter": N2}
for fused in (0, 1):
    x = torch.full((M, K), float("nan"), device=dev)
    c16 = torch.zeros(((M + 15) // 16 * 16) * N2, dtype=torch.float16, device=dev)

    def call(st=None):
        return f(Ap.data_ptr(), W1.data_ptr(), x.data_ptr(), g.data_ptr(), b.data_ptr(), W2.data_ptr(),
                 b2.data_ptr(), c16.data_ptr(), M, K, K, N2, sync.data_ptr(), fused, st)
    llm_capi.check(call(), lib)
    torch.cuda.synchronize()
    outs[fused] = (x.clone(), c16.clone())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(args.reps):
            call(st)
    gr.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / args.reps
        best = t if best is None else min(best, t)
    res["fused" if fused else "two_launches"] = round(best, 2)
    assert int(sync[2].item()) == 0, "arrival wait timed out"
    assert int(sync[0].item()) == 0 and int(sync[1].item()) == 0, sync
assert torch.equal(outs[0][0], outs[1][0]), "o_proj output differs"
assert torch.equal(outs[0][1].view(torch.int16), outs[1][1].view(torch.int16)), "fc1 output differs"
res["bitwise_equal"] = True
print(json.dumps(res))
