"""Per-layer timeline of an overlap-mode step (LLM_OVERLAP) from a rocprofv3
kernel trace: the attention launches (pa_split_kernel) on one queue, the
chain kernels on the other; for each attention launch its duration and the
chain busy time inside it, and the gaps where the attention queue waited.
    python scripts/overlap_timeline.py gpurun_out/trace_X/tr_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
adv = sorted([r for r in rows if "argmax_partials_kernel" in r["Kernel_Name"]], key=lambda r: r["e"])
t_beg, t_end = adv[-2]["e"], adv[-1]["e"]
step = [r for r in rows if r["s"] >= t_beg and r["e"] <= t_end]
att = [r for r in step if "pa_split_kernel" in r["Kernel_Name"]]
oth = [r for r in step if "pa_split_kernel" not in r["Kernel_Name"]]
t0 = step[0]["s"]
print(f"step span {(step[-1]['e'] - t0) / 1e3:.1f} us (to last start+), kernels {len(step)}, "
      f"attention {len(att)} ({sum(r['e'] - r['s'] for r in att) / 1e3:.1f} us busy), "
      f"other {len(oth)} ({sum(r['e'] - r['s'] for r in oth) / 1e3:.1f} us busy)")
prev_end = t0
gap_tot = 0
for i, a in enumerate(att):
    inside = sum(min(r["e"], a["e"]) - max(r["s"], a["s"]) for r in oth
                 if r["e"] > a["s"] and r["s"] < a["e"])
    gap = a["s"] - prev_end
    gap_tot += max(gap, 0)
    if i < 6 or i >= len(att) - 4:
        print(f"  att {i:3d} start {(a['s'] - t0) / 1e3:9.1f} dur {(a['e'] - a['s']) / 1e3:7.1f} "
              f"gap-before {gap / 1e3:7.1f}  chain busy inside {inside / 1e3:7.1f} us")
    prev_end = a["e"]
print(f"attention-queue idle between launches {gap_tot / 1e3:.1f} us; "
      f"tail after last attention {(step[-1]['e'] - att[-1]['e']) / 1e3:.1f} us")
# chain segments between consecutive attention ends: duration of the chain work
