#!/bin/bash
# Round 5: (a) one column tile per GEMM workgroup at <= 16 rows (pick_nt),
# (b) beam rows quantised by the o_proj prologue from fp32 pa_merge_kernel
# rows instead of pa_merge_row_kernel, against ab_base/ (the head before):
# the whole GPU suite, then same-box A/B at C3's 8 / 16-row points and C4.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/nt
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS=c4 ROUNDS=2 bash scripts/gpu_lib_ab.sh || exit 1
for B in 8 16; do
  AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch $B" bash scripts/gpu_lib_ab.sh | sed "s/^/rows $B: /" || exit 1
done
echo done
