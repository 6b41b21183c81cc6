#!/bin/bash
# fc1-output quantiser folded into fc2's prologue (in-tree A/B build) vs the
# quantiser launch (ab_old/): decoder parity, then C3 / C4 same-box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fc2qpro
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c3 c4" ROUNDS=2 STEPS=20 bash scripts/gpu_lib_ab.sh
