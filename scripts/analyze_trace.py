"""Timeline of one decode step from a rocprofv3 kernel trace: per-kernel-kind
busy time, overlap between queues, idle gaps.
    python scripts/analyze_trace.py gpurun_out/trace_X/tr_kernel_trace.csv [--dump]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
# the step's last kernel: the greedy argmax (which also advances the positions)
adv = [r for r in rows if "argmax_partials_kernel" in r["Kernel_Name"]]
nmb = len({r["Queue_Id"] for r in adv}) or 1
adv.sort(key=lambda r: r["e"])
t_end = adv[-1]["e"]
t_beg = adv[-1 - nmb]["e"] if len(adv) > nmb else rows[0]["s"]
step = [r for r in rows if r["s"] >= t_beg and r["e"] <= t_end]
t0 = step[0]["s"]
t1 = max(r["e"] for r in step)
print(f"step kernels {len(step)} span {(t1 - t0) / 1e3:.1f} us, queues {sorted({r['Queue_Id'] for r in step})}")
kind = defaultdict(float)
cnt = defaultdict(int)
by_grid = "--by-grid" in sys.argv  # split each kernel kind by its grid (GEMM shapes)
for r in step:
    k = re.sub(r"^void |llm::|\(.*$", "", r["Kernel_Name"])[:60]
    if by_grid:
        g = [r.get(c, "") for c in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size")]
        k = f"{k} grid={'x'.join(x for x in g if x)} wg={r.get('Workgroup_Size_X', r.get('Workgroup_Size', ''))}"
    kind[k] += (r["e"] - r["s"]) / 1e3
    cnt[k] += 1
for k, v in sorted(kind.items(), key=lambda kv: -kv[1]):
    print(f"  {v:9.1f} us  {cnt[k]:4d}x  avg {v / cnt[k]:7.2f}  {k}")
# union busy time
ev = sorted([(r["s"], 1) for r in step] + [(r["e"], -1) for r in step])
busy = 0
act = 0
last = None
multi = 0
for t, d in ev:
    if last is not None:
        if act > 0:
            busy += t - last
        if act > 1:
            multi += t - last
    act += d
    last = t
print(f"busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us, >1 kernel running {multi / 1e3:.1f} us")
if "--by-position" in sys.argv:
    # kernels per layer from the step's repeating pattern: position j of each
    # layer (o_proj and fc2 share a grid; this separates them)
    names = [re.sub(r"^void |llm::|\(.*$", "", r["Kernel_Name"])[:40] for r in step]
    per = int(sys.argv[sys.argv.index("--by-position") + 1])
    body = step[: (len(step) // per) * per]
    for j in range(per):
        ds = sorted((r["e"] - r["s"]) / 1e3 for r in body[j::per])
        g = "x".join(body[j].get(c, "") for c in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z") if body[j].get(c))
        print(f"  pos {j}: median {ds[len(ds) // 2]:7.2f} us  min {ds[0]:7.2f}  n {len(ds)}  {names[j]} grid={g}")
if "--dump" in sys.argv:
    for r in step[:80]:
        print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:70]}")
