"""Time the FP16 decode GEMMs (CUDADecoder, C2 shapes: hid 768, M = 16) per
(column tiles, waves, rows) form, graph-replayed so host launch cost is
excluded; every form is checked against the default launch.
    python scripts/tune_gemm_f16.py [--M 16] [--hid 768] [--reps 50]"""
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
ap.add_argument("--M", type=int, default=16)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--hid", type=int, default=768)
args = ap.parse_args()
lib = llm_capi.load_tune()
lib.f16_gemm_tune.restype = ctypes.c_int
lib.f16_gemm_tune.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                   ctypes.c_void_p] + [ctypes.c_int] * 3 + \
    [ctypes.c_void_p]
M, hid = args.M, args.hid
s = torch.cuda.Stream()
for name, K, N in [("o_proj", hid, hid), ("mlp_fc2", 4 * hid, hid), ("qkv_proj", hid, 3 * hid),
                   ("mlp_fc1", hid, 4 * hid)]:
    W = (torch.randn((K, N), device="cuda") * 0.05).half()
    copies = [llm_capi.pack_weights(W, llm_capi.LLM_F16) for _ in range(8)]
    A = (torch.randn((M, K), device="cuda")).half()
    Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_F16)
    C = torch.empty((M, N), device="cuda")
    ref = torch.empty_like(C)
    llm_capi.check(lib.f16_gemm_tune(0, 0, 0, 1, Ap.data_ptr(), K, copies[0].data_ptr(),
                                     ref.data_ptr(), M, N, K, None), lib)
    torch.cuda.synchronize()
    for nt in (1, 2):
        for w in (4, 8):
            for mr in (16, 32):
                if mr > 16 and M <= 16:
                    continue
                C.zero_()
                llm_capi.check(lib.f16_gemm_tune(nt, w, mr, 1, Ap.data_ptr(), K,
                                                 copies[0].data_ptr(), C.data_ptr(), M, N, K,
                                                 None), lib)
                torch.cuda.synchronize()
                assert torch.allclose(C, ref, rtol=1e-5, atol=1e-5), (name, nt, w, mr)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    st = torch.cuda.current_stream().cuda_stream
                    for r in range(args.reps):
                        lib.f16_gemm_tune(nt, w, mr, 1, Ap.data_ptr(), K, copies[r % 8].data_ptr(),
                                          C.data_ptr(), M, N, K, ctypes.c_void_p(st))
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / (3 * args.reps) * 1e3
                print(json.dumps({"gemm": name, "M": M, "K": K, "N": N, "NT": nt, "waves": w,
                                  "mrows": mr, "us": round(t, 2)}), flush=True)
