#!/bin/bash
# Kernel-level (rocprofv3 kernel trace) timing of the attention split launch
# per pages-per-split value at one shape (host launch overhead excluded):
#   SHAPE="--B 16 --H 12 --D 64 --T 2048" PPS="0 8 16 32" bash scripts/gpu_pps_trace.sh
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pps_trace
mkdir -p $O
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O -o pps -- python3 $R/scripts/sweep_attention_pps.py ${SHAPE:---B 16 --H 12 --D 64 --T 2048} --pps ${PPS:-0 8 16 32 64} --rounds 1 --iters 20 > $O/sweep.log 2>&1 || exit 1
cat $O/sweep.log | grep pps
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
g = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "pa_split" in n or "merge" in n:
        key = (n.split("(")[0][-40:], r.get("Grid_Size_X", r.get("Grid_Size", "")))
        g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in g.items():
    v = sorted(v)
    print(k, "n", len(v), "median us", round(v[len(v) // 2], 2))
PY
