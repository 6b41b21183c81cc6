"""Byte attribution of the decode GEMM forms (scripts/gpu_r3_gemm_attr.sh):
per form, the median per-dispatch L2 fetch bytes (2 x FETCH_SIZE, the gfx950
correction of MI355X_MICROARCH.md) and write bytes (WRITE_SIZE), against a
model of what each L2 must fetch:

  weights  K*N once (a column tile's row blocks share an XCD: linear
           workgroup id x + gx*y with gx % 8 == 0 keeps them on XCD x % 8)
  A        M*K per XCD that runs a workgroup needing it: all 8 XCDs without
           the XCD placement, 8 / slices XCDs per slice with it (each XCD's L2
           fetches A from the Infinity Cache or HBM on its own)
  output   slices * M * N * 4 (int32) written

    python scripts/gemm_attr_summarize.py OUT_DIR plan.json > summary.json"""
import csv
import json
import sys
from pathlib import Path


def dispatches(d, counters):
    out = {}
    for f in Path(d).rglob("*kernel_trace.csv" if not counters else "*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "gemm_kernel" not in r["Kernel_Name"]:
                    continue
                i = int(r["Dispatch_Id"])
                e = out.setdefault(i, {})
                if counters:
                    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                else:
                    e["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    return [out[i] for i in sorted(out)]


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    d = Path(sys.argv[1])
    plan = json.loads(Path(sys.argv[2]).read_text())
    tr = dispatches(d / "trace", False)
    fe = dispatches(d / "fetch", True)
    wr = dispatches(d / "write", True)
    res = []
    i = 0
    for p in plan:
        n = p["iters"]
        M, K, N, ks = p["M"], p["K"], p["N"], p["kslices"]
        sl = slice(i + 1, i + n)  # the first launch of a form warms the code object
        i += n
        w_bytes = K * N
        a_bytes = M * K
        a_mult = 8 / ks if p["xcd_map"] else 8
        out_bytes = ks * M * N * 4
        fetch = med([2 * 1024 * e.get("FETCH_SIZE", 0) for e in fe[sl]])
        write = med([1024 * e.get("WRITE_SIZE", 0) for e in wr[sl]])
        us = med([e["us"] for e in tr[sl]])
        model = w_bytes + a_mult * a_bytes
        res.append({**{k: p[k] for k in ("gemm", "M", "K", "N", "NT", "waves", "mrows", "kslices",
                                          "xcd_map")},
                    "us": round(us, 2),
                    "weights_B": w_bytes, "A_B": a_bytes, "A_fetch_mult_model": a_mult,
                    "out_B": out_bytes,
                    "fetch_B_pmc": int(fetch), "fetch_B_model": int(model),
                    "fetch_pmc_over_model": round(fetch / model, 3),
                    "write_B_pmc": int(write), "write_pmc_over_out": round(write / out_bytes, 3),
                    "pmc_over_unique": round((fetch + write) / (w_bytes + a_bytes + out_bytes), 3),
                    "weight_GBps": round(w_bytes / us / 1e3, 1)})
    print(json.dumps({"note": "L2 fetch bytes = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; "
                              "model: weights once + A once per XCD that needs it",
                      "forms": res}, indent=1))


if __name__ == "__main__":
    main()
