#!/bin/bash
# Round-5 evidence session: per config (PROFILE_CONFIGS, default c3 c4 c2) a
# rocprofv3 kernel trace of bench.py (stats + per-kernel step timeline), then
# the PMC traffic passes of the decoder's own attention launch (PMC_CONFIGS).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05prof
mkdir -p $O
for c in ${PROFILE_CONFIGS:-c3 c4 c2}; do
  bash $R/scripts/trace_step.sh r05_$c --config $c || { echo "trace $c failed"; tail -5 $R/gpurun_out/trace_r05_$c/bench.err; exit 1; }
  f=$(ls $R/gpurun_out/trace_r05_$c/*/*kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find $R/gpurun_out/trace_r05_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/analyze_trace.py $f --by-grid > $O/step_timeline_$c.txt || exit 1
  s=$(find $R/gpurun_out/trace_r05_$c -name "*kernel_stats.csv" | head -1)
  cp $s $O/kernel_stats_$c.csv
  head -14 $O/step_timeline_$c.txt
done
for c in ${PMC_CONFIGS:-}; do
  DEC=--decoder timeout -k 10 600 bash $R/scripts/gpu_pmc.sh $c || { echo "pmc $c failed"; exit 1; }
  cp $R/gpurun_out/pmc_attention_$c.json $O/
done
echo profiles done
