#!/bin/bash
# Round 5: fc2 at <= 16 INT8 rows as two k slices adding into x (fp32
# atomics, x zeroed by the LN2 launch) against ab_base/: the whole GPU suite,
# then same-box A/B at C3's 8 / 16-row points and C3 / C4 (unchanged paths).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/fc2k2
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for B in 8 16; do
  AB_DIR=ab_base CONFIGS=c3 ROUNDS=3 STEPS=20 EXTRA="--global-batch $B" bash scripts/gpu_lib_ab.sh | sed "s/^/rows $B: /" || exit 1
done
AB_DIR=ab_base CONFIGS="c3 c4" ROUNDS=1 STEPS=20 bash scripts/gpu_lib_ab.sh || exit 1
bash scripts/trace_step.sh r05k2_b8 --config c3 --global-batch 8 || exit 1
f=$(find gpurun_out/trace_r05k2_b8 -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py $f --by-grid > $O/step_timeline_c3_b8.txt && head -12 $O/step_timeline_c3_b8.txt
echo done
