"""Split-K forms of the decode GEMMs that feed a LayerNorm (o_proj, mlp_fc2):
column tiles per workgroup x waves x rows per workgroup x k slices x
XCD-aware slice placement (GemmArgs::xcd_map), graph-replayed over distinct
weight copies (past the 256 MiB Infinity Cache, as in the C3 step).  Every
form's slices are summed and checked against torch's int32 product first.
    python scripts/tune_gemm_sk.py [--M 64] [--reps 40]"""
import argparse
import ctypes
import itertools
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=64)
ap.add_argument("--reps", type=int, default=40)
ap.add_argument("--hid", type=int, default=2048)
ap.add_argument("--cache-bytes", type=float, default=320e6)
ap.add_argument("--only", default="")
args = ap.parse_args()
lib = llm_capi.load_tune()
lib.i8_gemm_tune_sk.restype = ctypes.c_int
lib.i8_gemm_tune_sk.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + \
    [ctypes.c_void_p]
M, hid = args.M, args.hid
shapes = [("o_proj", hid, hid), ("mlp_fc2", 4 * hid, hid)]
s = torch.cuda.Stream()
torch.manual_seed(0)

for name, K, N in shapes:
    if args.only and name != args.only:
        continue
    W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
    Wp = llm_capi.pack_weights(W, llm_capi.LLM_I8)
    ncopies = max(2, int(args.cache_bytes // (K * N)) + 1)
    copies = [Wp.clone() for _ in range(ncopies)]
    A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda")
    Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_I8)  # A-fragment order
    ref = (A.double() @ W.double()).round().to(torch.int64).cpu()
    part = torch.empty((8, M, N), dtype=torch.int32, device="cuda")
    forms = [(nt, w, mr, ks, x) for nt, w, mr, ks, x in itertools.product(
        (1, 2, 4), (4, 8), (16, 32, 64), (1, 2, 4, 8), (0, 1))
        if not (x and ks == 1) and (K // 64) // ks >= 2 and mr <= 2 * M]
    for nt, w, mr, ks, x in forms:
        part.zero_()
        llm_capi.check(lib.i8_gemm_tune_sk(nt, w, mr, ks, x, Ap.data_ptr(), Wp.data_ptr(),
                                           part.data_ptr(), M, N, K, None))
        torch.cuda.synchronize()
        got = part[:ks].to(torch.int64).sum(0).cpu()
        assert torch.equal(got, ref), (name, nt, w, mr, ks, x)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            st = torch.cuda.current_stream().cuda_stream
            for r in range(args.reps):
                lib.i8_gemm_tune_sk(nt, w, mr, ks, x, Ap.data_ptr(), copies[r % ncopies].data_ptr(),
                                    part.data_ptr(), M, N, K, ctypes.c_void_p(st))
        g.replay()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / args.reps * 1e-3
            best = t if best is None else min(best, t)
        print(json.dumps({"gemm": name, "M": M, "K": K, "N": N, "NT": nt, "waves": w, "mrows": mr,
                          "kslices": ks, "xcd_map": x, "us": round(best * 1e6, 2),
                          "weight_GBps": round(K * N / best / 1e9, 1)}), flush=True)
        del g
