#!/bin/bash
# HISTORICAL (round 3): LLM_PREFETCH and its prefetch_lines_kernel graph branch existed only
# for this A/B and were removed after it (profiles/r03/prefetch_branch_ab.txt).
# Weight-prefetch side branch: bench arms per config, then a kernel trace of
# the best arm (per-GEMM times with prefetched weights).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pf
mkdir -p $O
export TMPDIR=/tmp
arm() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], d['ms_per_step_median_hip_events'])"
}
for c in ${CONFIGS:-c4 c2 c3}; do
  for rep in 1 2; do
    for b in 0 64 256; do arm ${c}_pf${b}_$rep $c LLM_PREFETCH=$b || exit 1; done
  done
done
for c in ${TRACE:-c4}; do
  LLM_PREFETCH=${TRACE_PF:-64} bash $R/scripts/trace_step.sh pf_$c --config $c || exit 1
  f=$(find $R/gpurun_out/trace_pf_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/analyze_trace.py $f --by-grid
done
