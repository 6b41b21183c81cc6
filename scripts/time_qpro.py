"""o_proj at C3 (64 rows, 2048 x 2048): packed int8 A (the merge launch's
output, i8_gemm_tune with the product tile) against fp32 rows quantised in
the GEMM's prologue (i8_gemm_tune_qpro), graph-replayed over distinct weight
copies; also checks the two give the same C (same quantisation).
    python scripts/time_qpro.py"""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

M, K, N, REPS = 64, 2048, 2048, 40
lib = llm_capi.load_tune()
lib.i8_gemm_tune_qpro.restype = ctypes.c_int
lib.i8_gemm_tune_qpro.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
lib.i8_gemm_tune.restype = ctypes.c_int
lib.i8_gemm_tune.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda")
W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
Wp = llm_capi.pack_weights(W, llm_capi.LLM_I8)
copies = [Wp.clone() for _ in range(80)]
sw = torch.rand(N, device="cuda") * 1e-2
# the merge launch's output: quantise_rows of x, packed
qr = torch.empty((M, K), dtype=torch.int8, device="cuda")
sa = torch.empty(M, device="cuda")
llm_capi.check(lib.quantize_rows(x.data_ptr(), M, K, qr.data_ptr(), sa.data_ptr(), None), lib)
torch.cuda.synchronize()
q = llm_capi.pack_weights(qr.t().contiguous(), llm_capi.LLM_I8)  # packed-A order
res = {}
for name in ("packed_int8", "qpro", "qpro_noprologue", "qpro_noprefetch"):
    C = torch.empty(M, N, device="cuda")

    def call(w, st=None):
        if name.startswith("qpro"):
            d = {"qpro": 0, "qpro_noprologue": 1, "qpro_noprefetch": 2}[name]
            return lib.i8_gemm_tune_qpro(x.data_ptr(), w.data_ptr(), C.data_ptr(), M, N, K, sw.data_ptr(), d, st)
        return lib.i8_gemm_tune(2, 8, 16, 1, q.data_ptr(), K, w.data_ptr(), C.data_ptr(), M, N, K,
                                sa.data_ptr(), sw.data_ptr(), st)
    llm_capi.check(call(Wp), lib)
    torch.cuda.synchronize()
    res[name + "_C"] = C.clone()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for r in range(REPS):
            call(copies[r % len(copies)], st)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
    res[name + "_us"] = round(best, 2)
print(json.dumps({k: v for k, v in res.items() if not k.endswith("_C")}))
print("same C:", torch.equal(res["packed_int8_C"], res["qpro_C"]))
