#!/bin/bash
# Kernel-level times of the D = 64 split-kernel variants at the C2 shape.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tune_c2
mkdir -p $O
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O -o t -- python3 $R/scripts/tune_attention_c2.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
g = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "pa_split_kernel<64" in n:
        args = n[n.index("<64"):n.index(">")+1]
        g[(args, r.get("Grid_Size_X", ""))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    v = sorted(v)
    print(k[1], k[0], "median us", round(v[len(v) // 2], 2))
PY
