"""Compare the GPU decoder's KV cache with the oracle's after N lockstep steps."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"),
                str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import llm_capi  # noqa: E402
import llm_decoder  # noqa: E402
from _util import rel_err  # noqa: E402
from oracle.oracle import Oracle, OracleDecoder, synthetic_int8_model  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def d2h(ptr, n, dtype):
    a = np.empty(n, dtype)
    assert hip.hipMemcpy(a.ctypes.data, ctypes.c_void_p(ptr), a.nbytes, 2) == 0
    return a


o = Oracle()
w = synthetic_int8_model(o, L=2, H=4, D=64, V=1000, max_seq=64, seed=1234)
c = w["cfg"]
B = 3
dec = llm_decoder.INT8Decoder(c["L"], c["H"], c["D"], c["hid"], c["V"], c["max_seq"], max_batch=B)
wd = {k: np.ascontiguousarray(v) for k, v in w.items() if k != "cfg"}
wd["emb"] = w["emb"].view(np.uint16)
dec.set_weights(wd)
odec = OracleDecoder(o, w, B)
dec.begin_synthetic(B, 0, 0, False)
logits = torch.empty((B, c["V"]), device="cuda")
rng = np.random.default_rng(0)
prompts = [list(rng.integers(0, 1000, n)) for n in (5, 17, 1)]
nxt = [0] * B
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 9
MODE = sys.argv[2] if len(sys.argv) > 2 else "greedy"
trng = np.random.default_rng(1)
SAVE = {7, 8}
saved = {}
lib = llm_capi.load()
for s in range(NS):
    tok = ([int(p[s]) if s < len(p) else nxt[b] for b, p in enumerate(prompts)] if MODE == "greedy"
           else [int(t) for t in trng.permutation(c["V"])[:B]])
    nxt = dec.step(tok, logits_ptr=logits.data_ptr())
    torch.cuda.synchronize()
    _, ol, _ = odec.step(np.array(tok, np.int32), np.full(B, s, np.int32))
    print("step", s, "tok", tok, "err per row", [f"{rel_err(logits.cpu().numpy()[b], ol[b]):.1e}" for b in range(B)])
    h = ctypes.c_void_p(dec.kv_handle)
    for l in range(c["L"]):
        v = llm_capi.PaKvView()
        llm_capi.check(lib.kv_cache_view(h, l, ctypes.byref(v)))
        TS, D, H = v.page_size, v.head_dim, v.num_heads
        both = d2h(v.k_pool, v.num_pages * 2 * TS * D, np.float16).reshape(v.num_pages, 2, TS, D)
        kp, vp = both[:, 0], both[:, 1]  # K / V pages interleave
        pt = d2h(v.page_table, v.num_beams * H * v.max_tiles, np.int32).reshape(v.num_beams, H, v.max_tiles)
        ok = o_k = odec.kv(l, 0)
        o_v = odec.kv(l, 1)
        nmis, kmax, vmax = 0, 0.0, 0.0
        for b in range(B):
            for t in range(s + 1):
                for hh in range(H):
                    page = pt[b, hh, t // TS]
                    gk, gv = kp[page, t % TS], vp[page, t % TS]
                    if not (np.array_equal(gk, o_k[b, hh, t]) and np.array_equal(gv, o_v[b, hh, t])):
                        nmis += 1
                        kmax = max(kmax, float(np.abs(gk.astype(np.float32) - o_k[b, hh, t]).max()))
                        vmax = max(vmax, float(np.abs(gv.astype(np.float32) - o_v[b, hh, t]).max()))
        print(f"   layer {l}: KV rows mismatched {nmis}, k maxdiff {kmax:.2e}, v maxdiff {vmax:.2e}")
        if s in SAVE:
            gk = np.stack([[[kp[pt[b, hh, t // TS], t % TS] for t in range(s + 1)] for hh in range(H)] for b in range(B)])
            gv = np.stack([[[vp[pt[b, hh, t // TS], t % TS] for t in range(s + 1)] for hh in range(H)] for b in range(B)])
            saved[f"k{l}_s{s}"] = gk
            saved[f"v{l}_s{s}"] = gv
    if s in SAVE:
        saved[f"tok_s{s}"] = np.array(tok, np.int32)
        saved[f"logits_s{s}"] = logits.cpu().numpy()
np.savez("gpurun_out/kv_dump.npz", **saved)
