"""Per-GEMM summary of scripts/gpu_gemm_pmc.sh: duration (kernel trace),
MFMA ops, MFMA busy cycles and HBM bytes per dispatch, against the gfx950
peaks (MI355X_MICROARCH.md: INT8 MFMA = 2x the BF16 rate, ~5 POPS dense;
HBM 8 TB/s).  The decoder is stepped eagerly, so the GEMM dispatches come in
layer order qkv, o_proj, fc1, fc2 (C3: M = 64 rows).

MFMA utilisation = SQ_INSTS_VALU_MFMA_MOPS_I8 * 512 ops / kernel duration /
peak, and cross-checked with SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (duration
* 2.4 GHz).  (rocprofv3's own MfmaUtil divides by GRBM_GUI_ACTIVE, which under
counter collection spans the serialised profiling window, ~10x the kernel.)

    python scripts/gemm_pmc_summarize.py gpurun_out/gemm_pmc > summary.json"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

PEAK_OPS = 5.0e15
PEAK_BW = 8.0e12
SIMDS = 1024
CLOCK = 2.4e9
M = 64
ROLES = ["qkv", "o_proj", "fc1", "fc2"]
SHAPES = {"qkv": (2048, 6144), "o_proj": (2048, 2048), "fc1": (2048, 8192), "fc2": (8192, 2048)}


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
        res[ROLES[j % 4]].append(e)
    return res


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    d = Path(sys.argv[1])
    tr = by_role(gemm_dispatches(d / "trace", "*kernel_trace.csv", False))
    cn = {s: by_role(gemm_dispatches(d / s, "*counter_collection.csv", True))
          for s in ("mfma", "mops", "fetch", "write")}
    res = {"config": "C3 INT8 decoder, 64 rows, eager steps (scripts/prof_gemm.py)",
           "peaks": {"int8_mfma_ops_per_s": PEAK_OPS, "hbm_bytes_per_s": PEAK_BW},
           "gemms": {}}
    tot_t = tot_w = 0.0
    for role in ROLES:
        K, N = SHAPES[role]
        t = med([e["dur"] for e in tr[role]])
        kern = tr[role][0]["kernel"] if tr[role] else None
        mops = med([e.get("SQ_INSTS_VALU_MFMA_MOPS_I8", 0) for e in cn["mops"][role]])
        busy = med([e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for e in cn["mfma"][role]])
        fetch = med([e.get("FETCH_SIZE", 0) for e in cn["fetch"][role]])
        write = med([e.get("WRITE_SIZE", 0) for e in cn["write"][role]]) if cn["write"][role] else None
        ops = 2.0 * M * K * N
        wbytes = K * N + 4 * N  # int8 weights + fp32 column scales
        ent = {"kernel": kern, "M": M, "K": K, "N": N, "dispatches": len(tr[role]),
               "median_us": round(t * 1e6, 2),
               "algorithmic_ops": ops,
               "mfma_ops_counted": mops * 512 if mops is not None else None,
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
        a_bytes = M * K + 4 * M
        out_b = M * (K * 4 + 2 * K * 2) if role == "qkv" else M * N * 4
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
                        "note": "M = 64 rows: 128 int8 ops per weight byte, far below the "
                                "~625 op/B ridge; these GEMMs are bounded by the weight "
                                "stream and launch latency, not by the MFMA pipes"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
