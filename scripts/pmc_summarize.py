"""Summarise rocprofv3 --pmc CSV output into per-kernel, per-dispatch counter
means, and (for the paged-attention launch) the HBM bytes per launch with the
gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half the
bytes of a 16-B-per-lane streaming read, so hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024.

    python scripts/pmc_summarize.py --fetch DIR1 --write DIR2 --algo-json ALGO.json \
        --out profiles/pmc_attention_c3.json
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def counters(d):
    """{kernel: {counter: mean value per dispatch}} over every counter CSV in d."""
    acc = defaultdict(lambda: defaultdict(list))
    for f in Path(d).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or "?"
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": max(map(len, cs.values()))}
            for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--algo-json", required=True, help="prof_attention.py output line")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f, w = counters(a.fetch), counters(a.write)
    algo = json.loads(Path(a.algo_json).read_text().strip().splitlines()[-1])
    kernels = {}
    for k in sorted(set(f) | set(w)):
        kernels[k] = {"FETCH_SIZE_KiB": f.get(k, {}).get("FETCH_SIZE"),
                      "WRITE_SIZE_KiB": w.get(k, {}).get("WRITE_SIZE"),
                      "dispatches": f.get(k, {}).get("dispatches")}
    hbm = 0.0
    for k, v in kernels.items():
        if "pa_split_kernel" in k or "pa_merge_kernel" in k or "pa_merge_row_kernel" in k:
            hbm += 2.0 * (v["FETCH_SIZE_KiB"] or 0.0) * 1024 + (v["WRITE_SIZE_KiB"] or 0.0) * 1024
    res = {"config": algo.get("config"), "pps": algo.get("pps"), "launch": algo.get("launch"),
           "nsplit": algo.get("nsplit"), "form": algo.get("form"),
           "algorithmic_bytes_per_launch": algo["algorithmic_bytes"],
           "hbm_bytes_per_launch": int(hbm),
           "traffic_over_algorithmic": round(hbm / algo["algorithmic_bytes"], 4),
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE reads 1/2 "
                         "of a 16-B/lane stream, MI355X_MICROARCH.md §HBM)",
           "kernels": kernels}
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "traffic_over_algorithmic")}))


if __name__ == "__main__":
    main()
