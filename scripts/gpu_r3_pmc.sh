#!/bin/bash
# Attention PMC (FETCH_SIZE / WRITE_SIZE) of the decoder's own launch at every
# benched config, plus the C3 GEMM PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  DEC=--decoder bash $R/scripts/gpu_pmc.sh $c || { echo "pmc $c failed"; exit 1; }
  cat $R/gpurun_out/att_algo_$c.json
done
[ "${SKIP_GEMM:-0}" = 1 ] || bash $R/scripts/gpu_gemm_pmc.sh
