#!/bin/bash
# Round 5: C5-width INT8 rows (hid 4096) merged in the attention workgroup
# into fp32 rows + one quantise launch, instead of split + pa_merge_row_kernel,
# against ab_base/: decoder / attention tests, then same-box A/B at C5 (and C3,
# C4, which must not move).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/c5wgm
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py tests/test_wg_merge_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|C5" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS="c5" ROUNDS=3 STEPS=20 bash scripts/gpu_lib_ab.sh || exit 1
AB_DIR=ab_base CONFIGS="c3 c4" ROUNDS=1 STEPS=20 bash scripts/gpu_lib_ab.sh || exit 1
echo done
