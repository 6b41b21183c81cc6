"""Launch the D = 64 split-kernel variants of pa_decode_tune (tuning build) at
the C2 attention shape (16 rows x 12 heads x 2048 tokens, interleaved K/V
pages in shuffled order) for a few pages-per-split values.  Run under
rocprofv3 --kernel-trace (scripts/gpu_tune_c2.sh) for kernel-level times."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

B, H, D, T, ts = 16, 12, 64, 2048, 16
nt = T // ts
n = B * H * nt
g = torch.Generator(device="cuda").manual_seed(0)
kv = torch.randn((2 * n + 1, ts, D), generator=g, device="cuda").half()
pt = (2 * torch.randperm(n, generator=g, device="cuda")).to(torch.int32).reshape(B, H, nt)
q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
lib = llm_capi.load_tune()
lib.pa_decode_tune.restype = ctypes.c_int
lib.pa_decode_tune.argtypes = [ctypes.c_int, ctypes.POINTER(llm_capi.PaKvView), ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_void_p]
view = llm_capi.kv_view(kv[:-1], kv[1:], pt)
out = torch.empty((B, H, D), device="cuda")
ws = torch.empty(B * H * 128 * (D + 2) * 4, dtype=torch.uint8, device="cuda")
ref = llm_capi.pa_decode(q, kv[:-1], kv[1:], pt, T=T)
for pps in (32, 16, 8):
    for v in (20, 21, 22, 23, 24, 25):
        for it in range(12):
            llm_capi.check(lib.pa_decode_tune(v, ctypes.byref(view), llm_capi.ptr(q),
                                              llm_capi.ptr(out), None, B, H, T, pps,
                                              llm_capi.ptr(ws), ws.numel(), None), lib)
        torch.cuda.synchronize()
        if v < 24:
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-5, (v, pps, err)
print("done", flush=True)
