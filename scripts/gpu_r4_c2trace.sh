#!/bin/bash
# Kernel traces of the C2 step with the in-tree library and with ab_old/ (same
# box), each summarised per kernel kind (scripts/analyze_trace.py --by-grid).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c2trace
mkdir -p $O
for v in new old; do
  if [ $v = old ]; then export LD_LIBRARY_PATH=$R/ab_old${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}; fi
  bash $R/scripts/trace_step.sh c2$v --config ${TRACE_CONFIG:-c2} || { echo "trace $v failed"; tail -5 $R/gpurun_out/trace_c2$v/bench.err; exit 1; }
  f=$(find $R/gpurun_out/trace_c2$v -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/analyze_trace.py $f --by-grid > $O/step_timeline_$v.txt || exit 1
  head -12 $O/step_timeline_$v.txt
done
