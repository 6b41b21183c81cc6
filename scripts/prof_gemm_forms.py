#!/usr/bin/env python3
"""Driver for the GEMM byte attribution (scripts/gpu_r3_gemm_attr.sh): the C3
o_proj and mlp_fc2 shapes (M = 64) in several tile / split-K / XCD-placement
forms of the tuning build (i8_gemm_tune_sk: int32 output), ITERS eager
launches per form in a fixed order, so rocprofv3's per-dispatch FETCH_SIZE /
WRITE_SIZE rows can be attributed to weights, A and output by the form's
geometry (scripts/gemm_attr_summarize.py).  Prints the form list as JSON."""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import torch  # noqa: E402

import llm_capi  # noqa: E402

ITERS = int(os.environ.get("ITERS", "6"))
M = 64
# (name, K, N); forms: (NT, waves, rows per workgroup, k slices, xcd placement)
SHAPES = [("o_proj", 2048, 2048), ("mlp_fc2", 8192, 2048)]
FORMS = [(2, 8, 16, 1, 0), (1, 8, 64, 2, 0), (1, 8, 64, 2, 1), (1, 8, 64, 8, 1), (2, 8, 64, 1, 0)]


def main():
    lib = llm_capi.load_tune()
    lib.i8_gemm_tune_sk.restype = ctypes.c_int
    lib.i8_gemm_tune_sk.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p]
    torch.cuda.set_device(0)
    plan = []
    for name, K, N in SHAPES:
        W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
        Wp = llm_capi.pack_weights(W, llm_capi.LLM_I8)
        A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda")
        Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_I8)
        part = torch.empty((8, M, N), dtype=torch.int32, device="cuda")
        # a 512 MiB sweep between launches: weights and A start outside L2 and
        # the Infinity Cache, as in the decode step (the KV scan in between)
        flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        for f in FORMS:
            for _ in range(ITERS):
                flush.fill_(1)
                llm_capi.check(lib.i8_gemm_tune_sk(*f, Ap.data_ptr(), Wp.data_ptr(), part.data_ptr(),
                                                   M, N, K, None), lib)
            plan.append({"gemm": name, "K": K, "N": N, "M": M, "NT": f[0], "waves": f[1],
                         "mrows": f[2], "kslices": f[3], "xcd_map": f[4], "iters": ITERS})
        torch.cuda.synchronize()
        del flush
    print(json.dumps(plan))


if __name__ == "__main__":
    main()
