"""The paged-attention launch inside the decode step against the same launch
run on its own (bench.py's time_attention: llm_decoder_run_attention of layer
0, 3 warm-up + 20 timed launches after the timed steps), from one rocprofv3
run of bench.py: kernel durations (--kernel-trace) and per-dispatch counters
(--pmc passes).  The last ALONE attention dispatches of the run are the
standalone ones, the earlier ones are in-step.

    python scripts/instep_vs_alone.py TRACE_DIR [PMC_DIR ...] [--alone 23] [--match pa_split_kernel]
"""
import argparse
import csv
from collections import defaultdict
from pathlib import Path

import numpy as np


def rows_of(d, pattern):
    out = []
    for f in Path(d).rglob(pattern):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pmc", nargs="*")
    ap.add_argument("--alone", type=int, default=23)
    ap.add_argument("--match", default="pa_split_kernel")
    a = ap.parse_args()
    tr = [r for r in rows_of(a.trace, "*kernel_trace.csv") if a.match in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr])
    n = len(dur)
    step, alone = dur[:n - a.alone], dur[n - a.alone:]
    print(f"{a.match}: {n} dispatches; in-step {len(step)} median {np.median(step):.2f} us "
          f"(p10 {np.percentile(step, 10):.2f}, p90 {np.percentile(step, 90):.2f}); alone "
          f"{len(alone)} median {np.median(alone):.2f} us (p10 {np.percentile(alone, 10):.2f}, "
          f"p90 {np.percentile(alone, 90):.2f})")
    for d in a.pmc:
        per = defaultdict(dict)
        names = {}
        for r in rows_of(d, "*counter_collection.csv"):
            if a.match not in r.get("Kernel_Name", ""):
                continue
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[r["Counter_Name"]] = 1
        ids = sorted(per)
        if not ids:
            print(f"{d}: no {a.match} dispatches")
            continue
        s_ids, a_ids = ids[:len(ids) - a.alone], ids[len(ids) - a.alone:]
        for c in sorted(names):
            sv = np.array([per[i].get(c, np.nan) for i in s_ids])
            av = np.array([per[i].get(c, np.nan) for i in a_ids])
            print(f"  {c:28s} in-step {np.nanmean(sv):14.1f}   alone {np.nanmean(av):14.1f}   "
                  f"ratio {np.nanmean(sv) / max(np.nanmean(av), 1e-9):.3f}")


if __name__ == "__main__":
    main()
