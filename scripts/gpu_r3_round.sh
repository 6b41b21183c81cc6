#!/bin/bash
# Cheaper exact int8 rounding (common.hpp quant_i8): parity tests, the
# standalone o_proj prologue timing, then a C3 / C4 same-box A/B (ab_old/).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py tests/test_pa_decode_gpu.py tests/test_c4_beams_gpu.py tests/test_pa_prefill_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 scripts/time_qpro.py | head -1
CONFIGS="c3 c4" ROUNDS=2 STEPS=20 bash scripts/gpu_lib_ab.sh
