#!/bin/bash
# Round 5: the <= 16-row LM head (lm_head_x1_kernel) with its first two E
# batches issued before x is staged, and 12-k-step batches when that covers K
# (C2, C1) against ab_base/: tests, then same-box A/B at C2, C1 and C3's 8 rows.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/lmx1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|lm_head" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS="c2 c1" ROUNDS=3 STEPS=50 bash scripts/gpu_lib_ab.sh || exit 1
AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch 8" bash scripts/gpu_lib_ab.sh | sed "s/^/rows 8: /" || exit 1
for sh in 16,50257,768 8,50257,2048 1,50257,256; do
  LM_SHAPE=$sh timeout -k 10 300 python scripts/time_lm_head.py 2>&1 | grep max_abs | sed "s/^/lm_head $sh: /" || exit 1
done
echo done
