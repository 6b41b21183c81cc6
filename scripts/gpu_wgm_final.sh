#!/bin/bash
# Workgroup-merge round, final: every GPU test, the C2 A/B (product vs the
# tuning build's split + merge launches) and a C2 step trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
SPLITS=3 bash scripts/gpu_wgm_splits.sh || exit 1
bash scripts/trace_step.sh c2 --config c2 || exit 1
python scripts/analyze_trace.py gpurun_out/trace_c2/tr_kernel_trace.csv > gpurun_out/trace_c2/timeline.txt 2>&1 || true
head -12 gpurun_out/trace_c2/timeline.txt
timeout -k 10 300 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -5 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
