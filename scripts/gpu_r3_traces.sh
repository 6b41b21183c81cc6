#!/bin/bash
# Kernel traces of the C2 / C4 / C3 steps with per-grid breakdown.
set -o pipefail
R=$GRAFT_REPO_ROOT
for c in ${CONFIGS:-c2 c4 c3}; do
  bash $R/scripts/trace_step.sh $c --config $c || { echo "trace $c failed"; tail -20 $R/gpurun_out/trace_$c/bench.err; exit 1; }
  f=$(find $R/gpurun_out/trace_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/analyze_trace.py $f --by-grid > $R/gpurun_out/trace_$c/analysis.txt && cat $R/gpurun_out/trace_$c/analysis.txt
done
