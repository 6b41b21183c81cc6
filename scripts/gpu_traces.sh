#!/bin/bash
# Kernel-trace the step of each named config and summarise one step's timeline.
#   bash scripts/gpu_traces.sh c3 c2 ...
set -o pipefail
R=$GRAFT_REPO_ROOT
for c in "$@"; do
  bash $R/scripts/trace_step.sh $c --config $c || { echo "trace $c failed"; tail -20 $R/gpurun_out/trace_$c/bench.err; exit 1; }
  f=$(find $R/gpurun_out/trace_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/analyze_trace.py $f > $R/gpurun_out/trace_$c/analysis.txt && cat $R/gpurun_out/trace_$c/analysis.txt
done
