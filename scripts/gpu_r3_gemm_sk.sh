#!/bin/bash
# Split-K / XCD-placement sweep of o_proj and mlp_fc2 (scripts/tune_gemm_sk.py) at C3 (64) and C4 (32) rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_sk
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u scripts/tune_gemm_sk.py --M 64 > $O/m64.jsonl 2> $O/m64.err || { tail -20 $O/m64.err; exit 1; }
timeout -k 10 400 python3 -u scripts/tune_gemm_sk.py --M 32 > $O/m32.jsonl 2> $O/m32.err || { tail -20 $O/m32.err; exit 1; }
python3 - <<'PY'
import json
for f in ("m64", "m32"):
    rows = [json.loads(l) for l in open(f"gpurun_out/gemm_sk/{f}.jsonl")]
    for g in ("o_proj", "mlp_fc2"):
        rs = sorted([r for r in rows if r["gemm"] == g], key=lambda r: r["us"])
        print(f, g, "best 8:")
        for r in rs[:8]:
            print("  ", r["us"], "NT", r["NT"], "w", r["waves"], "mr", r["mrows"], "ks", r["kslices"], "xcd", r["xcd_map"])
PY
