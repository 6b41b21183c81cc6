#!/bin/bash
# HISTORICAL: the persistent kernel and tests/test_wgm_persist_gpu.py were removed after this
# measurement (profiles/r03/wgm_persist_ab.txt); kept as the record of how it was run.
# Persistent workgroup-merge attention: parity (bitwise vs one workgroup per
# item, and the WGM / decoder suites), then a same-box C3 A/B against the
# previous product library in ab_old/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/persist
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_wgm_persist_gpu.py tests/test_wg_merge_gpu.py tests/test_decoder_long_context_gpu.py tests/test_c3_properties_gpu.py tests/test_decoder_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c3" ROUNDS=3 STEPS=30 bash scripts/gpu_lib_ab.sh
