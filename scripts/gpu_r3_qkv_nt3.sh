#!/bin/bash
# HISTORICAL: the product rule it measured was reverted (profiles/r03/gemm_nt3_ab.txt).
# C3 qkv as 3 column tiles x 32 rows (narrow_tile_for): GEMM exactness, the
# teacher-forced hidden-2048 decoder tests (40 / 48 rows take the new form,
# KV append included), C3 properties, then a same-box C3 A/B against the
# previous product library in ab_old/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/nt3
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_decoder_gpu.py tests/test_c3_properties_gpu.py tests/test_decoder_long_context_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c3" ROUNDS=3 STEPS=30 bash scripts/gpu_lib_ab.sh
