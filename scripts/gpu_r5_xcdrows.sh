#!/bin/bash
# Round 5: one-workgroup-per-row kernels that write packed-A rows (merge_row,
# LayerNorm, the fc1 quantiser) with rows 8x..8x+7 on XCD x, so each 128-byte
# line of a fragment is written from one L2, against ab_base/ (the head
# before): the whole GPU suite, then same-box A/B at C4, C3 and 8 rows.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/xcdrows
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS="c4 c3" ROUNDS=2 STEPS=20 bash scripts/gpu_lib_ab.sh || exit 1
AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch 8" bash scripts/gpu_lib_ab.sh | sed "s/^/rows 8: /" || exit 1
bash scripts/trace_step.sh r05x_c4 --config c4 || exit 1
f=$(find gpurun_out/trace_r05x_c4 -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py $f --by-grid > $O/step_timeline_c4.txt && head -12 $O/step_timeline_c4.txt
echo done
