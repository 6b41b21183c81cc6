#!/bin/bash
# Round 5: fp32-row launches of exactly one resident round with > 8 splits
# (C3's model at 8 rows per GPU) run half the splits, twice as long; this tree
# vs ab_base/: decoder / attention tests, then same-box A/B at 8 rows.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/half
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py tests/test_pa_decode_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS=c3 ROUNDS=3 STEPS=20 EXTRA="--global-batch 8" bash scripts/gpu_lib_ab.sh | sed "s/^/rows 8: /" || exit 1
echo done
