"""Time the decode GEMMs (C3 shapes, M = 64) per column-tile variant, with
launches captured in a torch CUDA graph so host launch cost is excluded.
    python scripts/tune_gemm.py [--M 64] [--reps 50]"""
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
ap.add_argument("--M", type=int, default=64)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--hid", type=int, default=2048)
ap.add_argument("--copies", type=int, default=8)
ap.add_argument("--nts", type=int, nargs="*", default=[1, 2])
ap.add_argument("--only", default="")
args = ap.parse_args()
lib = llm_capi.load_tune()  # tuning build: `make tune`
lib.i8_gemm_tune.restype = ctypes.c_int
lib.i8_gemm_tune.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p] + \
    [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
M, hid = args.M, args.hid
shapes = [("qkv_proj", hid, 3 * hid), ("o_proj", hid, hid), ("mlp_fc1", hid, 4 * hid),
          ("mlp_fc2", 4 * hid, hid)]
s = torch.cuda.Stream()

for name, K, N in shapes:
    if args.only and name not in args.only.split(","):
        continue
    W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
    Wp = llm_capi.pack_weights(W, llm_capi.LLM_I8)
    # distinct weight copies so consecutive launches stream from HBM, not L2/MALL
    # (--copies 64: past the 256 MB Infinity Cache, as in the decode step)
    copies = [Wp.clone() for _ in range(args.copies)]
    A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda")
    sa = torch.rand(M, device="cuda")
    sw = torch.rand(N, device="cuda")
    C = torch.empty((M, N), device="cuda")
    ref = torch.empty_like(C)
    Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_I8)  # A-fragment order
    llm_capi.check(lib.i8_gemm_tune(1, 8, 0, 0, A.data_ptr(), K, Wp.data_ptr(),
                                    ref.data_ptr(), M, N, K, sa.data_ptr(), sw.data_ptr(), None))
    grid = [(nt, w, 1, mr) for nt in args.nts for w in (4, 8) for mr in (16, 32, 64)
            if mr >= 16 * ((M + 63) // 64) or mr < M or mr == 16]
    for nt, ks, apk, mr in grid:
        for _ in range(1):
            C.zero_()
            llm_capi.check(lib.i8_gemm_tune(nt, ks, mr, apk, (Ap if apk else A).data_ptr(), K,
                                            Wp.data_ptr(),
                                            C.data_ptr(), M, N, K, sa.data_ptr(), sw.data_ptr(),
                                            None))
            torch.cuda.synchronize()
            assert torch.equal(C, ref), (name, nt, ks)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            st = torch.cuda.current_stream().cuda_stream
            for r in range(args.reps):
                lib.i8_gemm_tune(nt, ks, mr, apk, (Ap if apk else A).data_ptr(), K,
                                 copies[r % len(copies)].data_ptr(),
                                 C.data_ptr(), M, N, K, sa.data_ptr(), sw.data_ptr(),
                                 ctypes.c_void_p(st))
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / (3 * args.reps) * 1e-3
        byts = K * N
        print(json.dumps({"gemm": name, "M": M, "K": K, "N": N, "NT": nt, "waves": ks, "a_packed": apk, "mrows": mr, "us": round(t * 1e6, 2),
                          "weight_GBps": round(byts / t / 1e9, 1)}), flush=True)
