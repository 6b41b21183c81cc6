#!/bin/bash
# Round-6 GPU session driver: each STEPS word runs one measured step into
# gpurun_out/r06/ (every step under its own time limit; the first failure ends
# the session).  STEPS="freerun tune probe bench" by default.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
O=gpurun_out/r06
for s in ${STEPS:-freerun tune probe bench}; do
  case $s in
    freerun)  # measurement: every test runs (no -x); a failure does not end the session
      timeout -k 10 900 python -u -m pytest tests/test_generate_free_run_gpu.py tests/test_decoder_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/free_run_tests.log 2>&1
      rc=$?; grep -E "FAILED|passed|failed" $O/free_run_tests.log | tail -8
      [ $rc -le 1 ] || exit $rc ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
      rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    tune)
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --copies 64 > $O/tune_gemm_c3.txt 2>&1 || exit 1
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --hid 4096 --copies 16 > $O/tune_gemm_c5.txt 2>&1 || exit 1 ;;
    probe)
      timeout -k 10 400 python -u scripts/overlap_probe.py > $O/overlap_probe.txt 2>&1 || { tail -20 $O/overlap_probe.txt; exit 1; }
      grep -E "^(base|xcd|four|bits)" $O/overlap_probe.txt || true ;;
    pmc*)  # GEMM MFMA utilisation + bytes, pmc<config> (default c3)
      c=${s#pmc}; c=${c:-c3}
      CFG=$c timeout -k 10 1000 bash scripts/gpu_gemm_pmc.sh || exit 1 ;;
    bench*)
      c=${s#bench}; c=${c:-c3}
      timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])" ;;
  esac
done
