#!/bin/bash
# HISTORICAL (round 3): the LLM_WKEEP / LLM_LMKEEP / LLM_DIAG_SKIP_FC1_QUANT switches existed
# only for this A/B and were removed after it; the winning policy is decoder.cpp w_keep_for
# (profiles/r03/wkeep_ab.txt).
# GEMM weight cache policy A/B (default policy = kept in the Infinity Cache vs nt).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wk
mkdir -p $O
export TMPDIR=/tmp
arm() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], d['ms_per_step_median_hip_events'])"
}
for rep in 1 2; do
  arm c2_k0_$rep c2 LLM_WKEEP=0 || exit 1
  arm c2_k1_$rep c2 LLM_WKEEP=1 || exit 1
  arm c2_k1lm_$rep c2 LLM_WKEEP=1 LLM_LMKEEP=1 || exit 1
  arm c4_k0_$rep c4 LLM_WKEEP=0 || exit 1
  arm c4_k1_$rep c4 LLM_WKEEP=1 || exit 1
  arm c1_k0_$rep c1 LLM_WKEEP=0 || exit 1
  arm c1_k1_$rep c1 LLM_WKEEP=1 || exit 1
done
LLM_WKEEP=1 bash $R/scripts/trace_step.sh wk_c2 --config c2 || exit 1
python3 $R/scripts/analyze_trace.py $(find $R/gpurun_out/trace_wk_c2 -name "*kernel_trace.csv" | head -1) --by-grid
# the upper bound of folding the fc1-output quantiser into a neighbour: the
# step with that launch removed outright (diagnostic: fc2 then reads stale A)
for rep in 1 2; do
  arm c4_q_$rep c4 || exit 1
  arm c4_noq_$rep c4 LLM_DIAG_SKIP_FC1_QUANT=1 || exit 1
  arm c3_q_$rep c3 || exit 1
  arm c3_noq_$rep c3 LLM_DIAG_SKIP_FC1_QUANT=1 || exit 1
done
