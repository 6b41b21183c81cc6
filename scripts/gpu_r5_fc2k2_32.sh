#!/bin/bash
# Round 5: the two-slice fc2 extended to 17..32 rows (32-row, 4-wave slices)
# against ab_base/ (two slices at <= 16 rows only): tests, then same-box A/B
# at C4 and C3's 32-row point.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/fc2k2_32
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py tests/test_c4_beams_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS=c4 ROUNDS=3 STEPS=30 bash scripts/gpu_lib_ab.sh || exit 1
AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch 32" bash scripts/gpu_lib_ab.sh | sed "s/^/rows 32: /" || exit 1
echo done
