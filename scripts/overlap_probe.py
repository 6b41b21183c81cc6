"""Can the decode step's weight-GEMM chain run BESIDE the attention scan?

C3's attention is HBM-bound (6.7 TB/s) and its GEMMs are latency-bound (fixed
costs, broadcast A reads).  With the 64 rows as two halves, half A's GEMM chain
(o_proj .. fc2, LN1, qkv of the next layer) has no dependency on half B's
attention.  This probe times, on CU-partitioned streams
(hipExtStreamCreateWithCUMask):
  * the C3 attention launch (64 rows, rotating over the 24 layers) alone, on
    all CUs and on the attention partition;
  * a chain of the four C3 weight GEMMs at 32 rows alone on the GEMM partition;
  * both issued together (attention on one partition, the chains on the other).
    python scripts/overlap_probe.py [--mm-cus 16] [--layout low|spread]
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))


def cu_mask(bits, ncu=256):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


class Masked:
    """A CU-masked HIP stream (hipExtStreamCreateWithCUMask) wrapped as a torch
    ExternalStream; destroyed on close (each layout makes only its own pair, so
    the runtime's hardware queues are never shared between masks)."""

    def __init__(self, hip, bits, ncu):
        import torch
        words = cu_mask(bits, ncu)
        arr = (ctypes.c_uint32 * len(words))(*words)
        self.hip, self.h = hip, ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(self.h), len(words), arr)
        assert rc == 0, rc
        self.s = torch.cuda.ExternalStream(self.h.value)

    def close(self):
        import torch
        torch.cuda.synchronize()
        self.hip.hipStreamDestroy(self.h)


def census(cen, st, blocks=2048, spin=2000):
    """{xcc: set of (se, sh, cu)} the stream's workgroups ran on."""
    import torch
    out = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    assert cen.census(ctypes.c_void_p(out.data_ptr()), blocks, spin,
                      ctypes.c_void_p(st.cuda_stream)) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().astype(np.int64).reshape(-1, 2)
    res = {}
    for xcc, hw in o:
        cu, sh, se = (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
        res.setdefault(int(xcc) & 15, set()).add((int(se), int(sh), int(cu)))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mm-cus", type=int, nargs="*", default=[8, 16, 32])
    ap.add_argument("--layouts", nargs="*", default=["low", "spread"])
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--layers", type=int, default=24)
    a = ap.parse_args()
    import torch
    import bench
    import llm_capi
    import llm_decoder
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    torch.cuda.set_device(0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    cfg = bench.CONFIGS["c3"]
    L, hid = cfg["L"], cfg["H"] * cfg["D"]
    dec = llm_decoder.INT8Decoder(L, cfg["H"], cfg["D"], hid, cfg["V"], cfg["T"] + 16,
                                  max_batch=cfg["B"], page_size=cfg["ts"])
    dec.set_weights(bench.make_weights(cfg, 1234))
    dec.begin_synthetic(cfg["B"], cfg["T"], 1234, True)
    s_all = torch.cuda.Stream()
    dec.step(list(range(cfg["B"])), stream=s_all.cuda_stream)
    torch.cuda.synchronize()
    # GEMM operands: one weight set per layer (1.2 GB: no Infinity-Cache reuse)
    shapes = [(hid, 3 * hid), (hid, hid), (hid, 4 * hid), (4 * hid, hid)]
    M = a.rows
    Ws = []
    for l in range(a.layers):
        Ws.append([llm_capi.pack_weights(torch.randint(-127, 128, (K, N), dtype=torch.int8,
                                                       device="cuda"), llm_capi.LLM_I8)
                   for K, N in shapes])
    As = {K: torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda") for K, _ in shapes}
    sa = torch.rand(M, device="cuda")
    sws = {N: torch.rand(N, device="cuda") for _, N in shapes}
    lib = llm_capi.load()
    Cs = {N: torch.empty((M, N), device="cuda") for _, N in shapes}

    def chain(l, st):
        for (K, N), W in zip(shapes, Ws[l]):
            llm_capi.check(lib.i8_gemm(llm_capi.ptr(As[K]), K, llm_capi.ptr(W), None,
                                       llm_capi.ptr(Cs[N]), M, N, K, llm_capi.ptr(sa),
                                       llm_capi.ptr(sws[N]), None, 0,
                                       ctypes.c_void_p(st.cuda_stream)))

    def run(att_st, mm_st, n_att, n_chain):
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        e_att = torch.cuda.Event(enable_timing=True)
        e_mm = torch.cuda.Event(enable_timing=True)
        first = att_st or mm_st
        ev0.record(first)
        for st in (att_st, mm_st):
            if st is not None and st is not first:
                st.wait_event(ev0)
        t0 = time.perf_counter()
        ci = 0
        for i in range(max(n_att, 1)):
            if att_st is not None and i < n_att:
                dec.run_attention(i % L, att_st.cuda_stream)
            if mm_st is not None:
                per = (n_chain + max(n_att, 1) - 1) // max(n_att, 1)
                for _ in range(per):
                    if ci < n_chain:
                        chain(ci % a.layers, mm_st)
                        ci += 1
        host = time.perf_counter() - t0
        if att_st is not None:
            e_att.record(att_st)
        if mm_st is not None:
            e_mm.record(mm_st)
        torch.cuda.synchronize()
        r = {"host_issue_ms": round(host * 1e3, 3)}
        if att_st is not None:
            r["att_ms"] = round(ev0.elapsed_time(e_att), 3)
        if mm_st is not None:
            r["mm_ms"] = round(ev0.elapsed_time(e_mm), 3)
        return r

    n_att, n_chain = L, 2 * L
    res = {"base_att_all_cus": run(s_all, None, n_att, 0)}
    res["base_att_all_cus_2"] = run(s_all, None, n_att, 0)
    res["base_chain_all_cus"] = run(None, s_all, 0, n_chain)
    print("base", json.dumps(res), flush=True)
    cen = ctypes.CDLL(str(ROOT / "scripts/micro/libcensus.so"))
    cen.census.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    # which mask bits land on which XCC: bits i = r (mod 8), and 32-bit words
    bit_xcc = {}
    for r in range(8):
        m = Masked(hip, [i for i in range(ncu) if i % 8 == r], ncu)
        c = census(cen, m.s)
        m.close()
        print(f"bits = {r} mod 8 -> xcc {sorted(c)} cus {sum(len(v) for v in c.values())}", flush=True)
        if len(c) == 1:
            for i in range(r, ncu, 8):
                bit_xcc[i] = next(iter(c))
    for w in range(ncu // 32):
        m = Masked(hip, list(range(32 * w, 32 * w + 32)), ncu)
        c = census(cen, m.s)
        m.close()
        print(f"bits {32 * w}..{32 * w + 31} -> xcc {sorted(c)} cus "
              f"{sum(len(v) for v in c.values())}", flush=True)
    if len(bit_xcc) != ncu:
        print("no per-XCC bit map (bits = r mod 8 did not land on one XCC each)", flush=True)
        bit_xcc = {i: i % 8 for i in range(ncu)}
    by_xcc = {x: [i for i in range(ncu) if bit_xcc[i] == x] for x in range(8)}
    layouts = {
        "xcd0_all": by_xcc[0],               # one whole XCD for the chains
        "xcd0_half": by_xcc[0][:len(by_xcc[0]) // 2],
        "xcd0_quarter": by_xcc[0][:len(by_xcc[0]) // 4],
        "four_per_xcd": [i for x in range(8) for i in by_xcc[x][:4]],
    }
    for key, mm_bits in layouts.items():
        att_bits = [b for b in range(ncu) if b not in set(mm_bits)]
        s_att, s_mm = Masked(hip, att_bits, ncu), Masked(hip, mm_bits, ncu)
        ca, cm = census(cen, s_att.s), census(cen, s_mm.s)
        res[key] = {
            "mm_cus": len(mm_bits),
            "census_att": {x: len(v) for x, v in sorted(ca.items())},
            "census_mm": {x: len(v) for x, v in sorted(cm.items())},
            "att_alone": run(s_att.s, None, n_att, 0),
            "chain_alone": run(None, s_mm.s, 0, n_chain),
            "both": run(s_att.s, s_mm.s, n_att, n_chain),
            "both_2": run(s_att.s, s_mm.s, n_att, n_chain),
        }
        s_att.close()
        s_mm.close()
        print(key, json.dumps(res[key]), flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
