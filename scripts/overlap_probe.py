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

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"))


def cu_mask(bits, ncu=256):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


def masked_stream(hip, bits):
    import torch
    words = cu_mask(bits)
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


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
    for layout in a.layouts:
        for k in a.mm_cus:
            if layout == "low":
                mm_bits = list(range(k))
            else:  # every (ncu / k)-th CU
                mm_bits = list(range(0, ncu, ncu // k))[:k]
            att_bits = [b for b in range(ncu) if b not in set(mm_bits)]
            s_att = masked_stream(hip, att_bits)
            s_mm = masked_stream(hip, mm_bits)
            key = f"{layout}_{k}"
            res[key] = {
                "att_alone": run(s_att, None, n_att, 0),
                "chain_alone": run(None, s_mm, 0, n_chain),
                "both": run(s_att, s_mm, n_att, n_chain),
                "both_2": run(s_att, s_mm, n_att, n_chain),
            }
            print(key, json.dumps(res[key]), flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
