#!/bin/bash
# Workgroup-merge (FP16 attention) round: its parity tests, a same-box C2 A/B
# against ab_old/ (the split + merge build) and a C2 step trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wg_merge_gpu.py tests/test_decoder_gpu.py tests/test_pa_decode_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/wgm_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/wgm_tests.log; exit 1; }
tail -2 gpurun_out/wgm_tests.log
CONFIGS="c2" ROUNDS=2 bash scripts/gpu_lib_ab.sh || exit 1
bash scripts/trace_step.sh c2 --config c2 || exit 1
python scripts/analyze_trace.py gpurun_out/trace_c2/tr_kernel_trace.csv > gpurun_out/trace_c2/timeline.txt 2>&1 || true
head -12 gpurun_out/trace_c2/timeline.txt
