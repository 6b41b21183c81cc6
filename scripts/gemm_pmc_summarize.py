"""Per-GEMM summary of scripts/gpu_gemm_pmc.sh: duration (kernel trace),
MFMA ops, MFMA busy cycles and HBM bytes per dispatch, against the gfx950
peaks (MI355X_MICROARCH.md: INT8 MFMA = 2x the BF16 rate, ~5 POPS dense;
HBM 8 TB/s).  The decoder is stepped eagerly, so the GEMM dispatches come in
layer order qkv, o_proj, fc1, fc2 (C3: M = 64 rows).

MFMA utilisation = SQ_INSTS_VALU_MFMA_MOPS_I8 * 512 ops / kernel duration /
peak, and cross-checked with SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (duration
* 2.4 GHz).  (rocprofv3's own MfmaUtil divides by GRBM_GUI_ACTIVE, which under
counter collection spans the serialised profiling window, ~10x the kernel.)

FP16 decoder (C2): SQ_INSTS_VALU_MFMA_MOPS_F16 against the dense FP16 peak
(~2.5 PF); its o_proj runs inside the attention launch, so three GEMMs per
layer (qkv, fc1, fc2).

    python scripts/gemm_pmc_summarize.py gpurun_out/gemm_pmc [c3|c5|c2] > summary.json"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

PEAK_BW = 8.0e12
SIMDS = 1024
CLOCK = 2.4e9
# config -> (rows, hidden, weight dtype, GEMMs per layer in dispatch order)
CONFIGS = {
    "c3": (64, 2048, "i8", ["qkv", "o_proj", "fc1", "fc2"]),
    "c5": (64, 4096, "i8", ["qkv", "o_proj", "fc1", "fc2"]),
    "c2": (16, 768, "f16", ["qkv", "fc1", "fc2"]),
}
PEAKS = {"i8": 5.0e15, "f16": 2.5e15}  # dense MFMA (MI355X_MICROARCH.md)
MOPS = {"i8": "SQ_INSTS_VALU_MFMA_MOPS_I8", "f16": "SQ_INSTS_VALU_MFMA_MOPS_F16"}
CFG = sys.argv[2] if len(sys.argv) > 2 else "c3"
M, HID, DT, ROLES = CONFIGS[CFG]
PEAK_OPS = PEAKS[DT]
SHAPES = {"qkv": (HID, 3 * HID), "o_proj": (HID, HID), "fc1": (HID, 4 * HID),
          "fc2": (4 * HID, HID)}


def gemm_dispatches(d, pat, counters):
    """[(dispatch_id, kernel, {counter: value} or duration)] of gemm kernels in order."""
    out = {}
    for f in Path(d).rglob(pat):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "gemm_kernel" not in r["Kernel_Name"]:
                    continue
                i = int(r["Dispatch_Id"])
                e = out.setdefault(i, {"kernel": r["Kernel_Name"]})
                if counters:
                    e[r["Counter_Name"]] = float(r["Counter_Value"])
                else:
                    e["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return [out[i] for i in sorted(out)]


def by_role(lst):
    res = defaultdict(list)
    for j, e in enumerate(lst):
        res[ROLES[j % len(ROLES)]].append(e)
    return res


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    d = Path(sys.argv[1])
    tr = by_role(gemm_dispatches(d / "trace", "*kernel_trace.csv", False))
    cn = {s: by_role(gemm_dispatches(d / s, "*counter_collection.csv", True))
          for s in ("mfma", "mops", "fetch", "write")}
    res = {"config": f"{CFG} ({DT} weights), {M} rows, eager steps (scripts/prof_gemm.py)",
           "peaks": {"int8_mfma_ops_per_s": PEAK_OPS, "hbm_bytes_per_s": PEAK_BW},
           "gemms": {}}
    tot_t = tot_w = 0.0
    for role in ROLES:
        K, N = SHAPES[role]
        t = med([e["dur"] for e in tr[role]])
        kern = tr[role][0]["kernel"] if tr[role] else None
        mops = med([e.get(MOPS[DT], 0) for e in cn["mops"][role]])
        busy = med([e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for e in cn["mfma"][role]])
        fetch = med([e.get("FETCH_SIZE", 0) for e in cn["fetch"][role]])
        write = med([e.get("WRITE_SIZE", 0) for e in cn["write"][role]]) if cn["write"][role] else None
        ops = 2.0 * M * K * N
        es = 1 if DT == "i8" else 2
        wbytes = K * N * es + (4 * N if DT == "i8" else 0)  # weights (+ fp32 column scales)
        ent = {"kernel": kern, "M": M, "K": K, "N": N, "dispatches": len(tr[role]),
               "median_us": round(t * 1e6, 2),
               "algorithmic_ops": ops,
               "mfma_ops_counted": mops * 512 if mops else None,
               "mfma_ops_counter": MOPS[DT],
               "achieved_TOPS": round(ops / t / 1e12, 1),
               "mfma_util_vs_peak": round(ops / t / PEAK_OPS, 4),
               "mfma_busy_frac_from_cycles": round(busy / SIMDS / (t * CLOCK), 4) if busy else None,
               "weight_bytes": wbytes,
               "weight_GBps": round(wbytes / t / 1e9, 1),
               "hbm_frac_vs_8TBps": round(wbytes / t / PEAK_BW, 4),
               "hbm_bytes_pmc": int(2 * fetch * 1024) if fetch else None}
        # attribution: weights once; A (int8 M x K + row scales) once per XCD
        # (every XCD runs workgroups of every row block); output fp32 (qkv: q
        # fp32 + K / V fp16 into the pages)
        a_bytes = M * K * es + (4 * M if DT == "i8" else 0)
        if role == "qkv":
            out_b = M * (K * 4 + 2 * K * 2)  # q fp32 + K / V fp16 into the pages
        elif DT == "f16" and role == "fc1":
            out_b = M * N * 2  # fc2's packed fp16 input
        else:
            out_b = M * N * 4
        ent["attribution"] = {
            "weights_B": wbytes, "A_B": a_bytes, "A_xcd_fetches": 8, "output_B": out_b,
            "fetch_model_B": wbytes + 8 * a_bytes,
            "fetch_pmc_over_model": round(2 * fetch * 1024 / (wbytes + 8 * a_bytes), 3) if fetch else None,
            "write_B_pmc": int(write * 1024) if write else None,
            "write_pmc_over_output": round(write * 1024 / out_b, 3) if write else None,
            "pmc_over_unique": round((2 * fetch + (write or 0)) * 1024 / (wbytes + a_bytes + out_b), 3)
            if fetch else None}
        res["gemms"][role] = ent
        tot_t += t
        tot_w += wbytes
    res["per_layer"] = {"gemm_us": round(tot_t * 1e6, 2), "weight_bytes": tot_w,
                        "weight_GBps": round(tot_w / tot_t / 1e9, 1),
                        "note": f"M = {M} rows: {2 * M // (1 if DT == 'i8' else 2)} ops per weight byte, far "
                                f"below the ~{int(PEAK_OPS / PEAK_BW)} op/B ridge; these GEMMs "
                                "are bounded by the weight stream and launch latency, not by "
                                "the MFMA pipes"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
