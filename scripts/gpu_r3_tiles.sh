#!/bin/bash
# Round 3: parity of the 33..64-row tile forms, GEMM form sweeps (qkv / fc1 at
# 64 and 32 rows, o_proj / fc2 at hid 4096), C3 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tiles
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_decoder_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --copies 24 > $O/g64.jsonl 2> $O/g64.err || { tail $O/g64.err; exit 1; }
timeout -k 10 300 python -u scripts/tune_gemm.py --M 32 --copies 24 > $O/g32.jsonl 2> $O/g32.err || { tail $O/g32.err; exit 1; }
timeout -k 10 400 python -u scripts/tune_gemm_sk.py --M 64 --hid 4096 > $O/sk4096.jsonl 2> $O/sk4096.err || { tail $O/sk4096.err; exit 1; }
python3 - <<'PY'
import json
for f in ("g64", "g32", "sk4096"):
    rows = [json.loads(l) for l in open(f"gpurun_out/tiles/{f}.jsonl")]
    for g in sorted({r["gemm"] for r in rows}):
        rs = sorted([r for r in rows if r["gemm"] == g], key=lambda r: r["us"])
        print(f, g, " | ".join(f'{r["us"]} NT{r["NT"]} w{r["waves"]} mr{r["mrows"]} ks{r.get("kslices", "-")} x{r.get("xcd_map", "-")}' for r in rs[:5]))
PY
timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
