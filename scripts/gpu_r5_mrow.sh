#!/bin/bash
# Round 5: pa_merge_row_kernel's packed-int8 path with one barrier (each wave
# takes the absmax of its merged heads in registers) against ab_base/:
# tests through merge_row, then same-box A/B at C4 and C5.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/mrow
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py tests/test_c4_beams_gpu.py tests/test_pa_decode_gpu.py tests/test_wg_merge_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS="c4 c5" ROUNDS=2 STEPS=20 bash scripts/gpu_lib_ab.sh || exit 1
echo done
