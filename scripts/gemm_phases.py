"""Phase timeline of one decode GEMM launch from in-kernel s_memrealtime stamps
(i8_gemm_stamps): workgroup start skew, k-loop (weight stream) end, wave end,
and the next kernel's start, all relative to the earliest workgroup start.
    python scripts/gemm_phases.py [--M 64]"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import llm_capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=64)
ap.add_argument("--hid", type=int, default=2048)
ap.add_argument("--diag", type=int, nargs="*", default=[0],
                help="0 full kernel, 1 no A loads, 2 no epilogue, 3 both")
args = ap.parse_args()
lib = llm_capi.load_tune()  # tuning build: `make tune`
lib.i8_gemm_stamps.restype = ctypes.c_int
lib.i8_gemm_stamps.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + \
    [ctypes.c_void_p] * 5
M, hid = args.M, args.hid
# the decode step's forms: hid 2048 (C3) o_proj / fc2 as 32-row blocks; hid 4096
# (C5, 256 column tiles) one 64-row block
nr = 64 if hid >= 4096 else 32
shapes = [("qkv_proj", hid, 3 * hid, 2, 64), ("o_proj", hid, hid, 1, nr),
          ("mlp_fc1", hid, 4 * hid, 2, 64), ("mlp_fc2", 4 * hid, hid, 1, nr)]
for (name, K, N, nt, mr), diag in [(sh, d) for sh in shapes for d in args.diag]:
    W = torch.randint(-128, 128, (K, N), dtype=torch.int8, device="cuda")
    copies = [llm_capi.pack_weights(W, llm_capi.LLM_I8) for _ in range(4)]
    A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda")
    Ap = llm_capi.pack_weights(A.t().contiguous(), llm_capi.LLM_I8)
    sa = torch.rand(M, device="cuda")
    sw = torch.rand(N, device="cuda")
    C = torch.empty((M, N), device="cuda")
    nwg = (N // 16 // nt) * ((M + mr - 1) // mr)
    st = torch.empty((nwg, 48), dtype=torch.int64, device="cuda")
    end = torch.empty(1, dtype=torch.int64, device="cuda")
    spans = []
    for rep in range(12):  # back-to-back launches; the last ones are measured
        st.fill_(0)
        llm_capi.check(lib.i8_gemm_stamps(nt, 8 | (diag << 8), mr, Ap.data_ptr(), copies[rep % 4].data_ptr(),
                                          C.data_ptr(), M, N, K, sa.data_ptr(), sw.data_ptr(),
                                          st.data_ptr(), end.data_ptr(), None))
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.int64)
        e = int(end.item())
        t0 = s[:, 0:8].min()
        start = (s[:, 0:8].min(axis=1) - t0) / 100.0  # us
        loop = (s[:, 16:24].max(axis=1) - t0) / 100.0
        wend = (s[:, 32:40].max(axis=1) - t0) / 100.0
        spans.append((start.max(), np.median(loop), loop.max(), wend.max(), (e - t0) / 100.0))
    a = np.array(spans[4:])
    print(f"{name:9s} diag {diag} wgs {nwg:4d}  last-wg-start {np.median(a[:, 0]):5.2f}  "
          f"k-loop done med {np.median(a[:, 1]):5.2f} max {np.median(a[:, 2]):5.2f}  "
          f"last wave end {np.median(a[:, 3]):5.2f}  next kernel {np.median(a[:, 4]):5.2f} us",
          flush=True)
