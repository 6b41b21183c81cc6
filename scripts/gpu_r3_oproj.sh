#!/bin/bash
# Fused o_proj (FP16 decoder): the parity tests that cover it, the C2 step
# timeline, then a same-box C2 A/B against the previous library (ab_old/,
# built from the last commit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/oproj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_wg_merge_gpu.py tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash $R/scripts/gpu_r3_oproj_trace.sh || exit 1
CONFIGS=${CONFIGS:-c2} ROUNDS=${ROUNDS:-2} bash scripts/gpu_lib_ab.sh
