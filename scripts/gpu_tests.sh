#!/bin/bash
# GPU parity tests only (optionally a subset: bash scripts/gpu_tests.sh tests/test_x.py ...).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | grep -v PASSED | head -40
tail -3 gpurun_out/gpu_tests.log
exit $rc
