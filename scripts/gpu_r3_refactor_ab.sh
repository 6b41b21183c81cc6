#!/bin/bash
# HISTORICAL: the device-function refactor it measured was reverted (profiles/r03/wgm_persist_ab.txt).
# After moving the split kernel body into a device function: parity of the
# workgroup-merge forms, then a same-box C3 / C2 A/B of the product library
# against the previous one in ab_old/, then the stage-size / occupancy sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/refactor
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_wgm_persist_gpu.py tests/test_wg_merge_gpu.py tests/test_pa_decode_gpu.py tests/test_c4_beams_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c3 c2" ROUNDS=2 STEPS=30 bash scripts/gpu_lib_ab.sh || exit 1
timeout -k 10 300 python scripts/tune_attention.py --interleave --rounds 5 --variants 1 3 6 8 9 5 > $O/stage_sweep.txt 2>&1 || exit 1
grep variant $O/stage_sweep.txt
