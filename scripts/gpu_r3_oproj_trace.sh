#!/bin/bash
# C2 step timeline with the fused o_proj (4 launches per layer).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/trace_step.sh c2 --config c2 || { tail -20 $R/gpurun_out/trace_c2/bench.err; exit 1; }
f=$(find $R/gpurun_out/trace_c2 -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/analyze_trace.py $f --by-grid --by-position ${PER:-4} > $R/gpurun_out/trace_c2/analysis.txt && cat $R/gpurun_out/trace_c2/analysis.txt
