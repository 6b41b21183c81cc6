#!/bin/bash
# Round-6 GPU session driver: each STEPS word runs one measured step into
# gpurun_out/r06/ (every step under its own time limit; the first failure ends
# the session).  STEPS="tests smoke bench" by default.  The round's experiment
# switches (LLM_OVERLAP, LLM_WGM_PARTS, LLM_FC2_K2_NT) were measured through
# "env:<VAR>=<v>:<config>" and removed with the code.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
O=gpurun_out/r06
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    t:*)  # t:<test file stem>[,<stem>...]: those GPU test files only
      f=""; for x in $(echo ${s#t:} | tr , ' '); do f="$f tests/$x.py"; done
      timeout -k 10 900 python -u -m pytest $f -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests_subset.log 2>&1
      rc=$?; grep -E "FAILED|ERROR" $O/tests_subset.log | head; tail -2 $O/tests_subset.log; [ $rc -eq 0 ] || exit $rc ;;
    freerun)  # measurement: every test runs (no -x); a failure does not end the session
      timeout -k 10 900 python -u -m pytest tests/test_generate_free_run_gpu.py tests/test_decoder_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/free_run_tests.log 2>&1
      rc=$?; grep -E "FAILED|passed|failed" $O/free_run_tests.log | tail -8
      [ $rc -le 1 ] || exit $rc ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
      rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    pmcatt*)  # pmcatt<config>: attention PMC traffic of the decoder's own launch
      c=${s#pmcatt}
      DEC=--decoder timeout -k 10 900 bash scripts/gpu_pmc.sh $c || exit 1
      python -c "import json;d=json.load(open('gpurun_out/pmc_attention_$c.json'));print('$c', {k: d[k] for k in list(d)[:8]})" ;;
    record*)  # record<config>: the full bench line (CPU baseline included) + the step's kernel trace
      c=${s#record}
      timeout -k 10 600 python bench.py --config $c > $O/r06_bench_$c.json 2> $O/r06_bench_$c.err || { tail -20 $O/r06_bench_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/r06_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'])"
      bash scripts/trace_step.sh $c --config $c || exit 1
      f=$(ls gpurun_out/trace_$c/*kernel_trace.csv | head -1)
      python scripts/analyze_trace.py $f --by-grid > $O/step_timeline_$c.txt && head -4 $O/step_timeline_$c.txt ;;
    tunent)  # the 3 / 4 column-tile forms (tuning build) at C3 and C5 shapes
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --copies 64 --nts 2 3 4 > $O/tune_gemm_nt_c3.txt 2>&1 || exit 1
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --hid 4096 --copies 16 --nts 2 3 4 > $O/tune_gemm_nt_c5.txt 2>&1 || exit 1 ;;
    tune)
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --copies 64 > $O/tune_gemm_c3.txt 2>&1 || exit 1
      timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --hid 4096 --copies 16 > $O/tune_gemm_c5.txt 2>&1 || exit 1 ;;
    probe)
      timeout -k 10 400 python -u scripts/overlap_probe.py > $O/overlap_probe.txt 2>&1 || { tail -20 $O/overlap_probe.txt; exit 1; }
      grep -E "^(base|xcd|four|bits)" $O/overlap_probe.txt || true ;;
    phases)  # in-kernel phase clocks of the GEMM forms (tuning build)
      for h in 2048 4096; do
        timeout -k 10 300 python -u scripts/gemm_phases.py --hid $h --diag 0 1 2 3 > $O/gemm_phases_$h.txt 2>&1 || { tail -5 $O/gemm_phases_$h.txt; exit 1; }
        grep diag $O/gemm_phases_$h.txt
      done ;;
    pmc*)  # GEMM MFMA utilisation + bytes, pmc<config> (default c3)
      c=${s#pmc}; c=${c:-c3}
      CFG=$c timeout -k 10 1000 bash scripts/gpu_gemm_pmc.sh || exit 1 ;;
    trace*)  # trace<config>: kernel trace of the bench step, per-kernel timeline
      c=${s#trace}; c=${c:-c3}
      bash scripts/trace_step.sh $c --config $c || exit 1
      f=$(ls gpurun_out/trace_$c/*kernel_trace.csv | head -1)
      python scripts/analyze_trace.py $f --by-grid | head -14 ;;
    ab*)  # ab<config>: same-box A/B of ab_base/ (scripts/build_ab_base.sh) against the tree
      c=${s#ab}; STEPS=30 AB_DIR=ab_base CONFIGS=$c ROUNDS=${ROUNDS:-2} timeout -k 10 1000 bash scripts/gpu_lib_ab.sh || exit 1 ;;
    env:*)  # env:<VAR>=<v>:<config>: bench line under that variable (A/B)
      v=${s#env:}; kv=${v%%:*}; c=${v#*:}
      env $kv timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/env_$c.json 2> $O/env_$c.err || { tail -20 $O/env_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/env_$c.json'));print('$kv $c',d['value'],d['ms_per_step'])" ;;
    tenv:*)  # tenv:<VAR>=<v>[+<VAR>=<v>...]:<config>: bench line on the TUNING build under those variables
      v=${s#tenv:}; kv=$(echo ${v%%:*} | tr + ' '); c=${v#*:}; tag=$(echo ${v%%:*} | tr -c 'A-Za-z0-9_\n' _)
      mkdir -p ab_tune && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so ab_tune/libllm_decoder_hip.so
      env $kv LD_LIBRARY_PATH=$PWD/ab_tune${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 400 python bench.py --config $c --steps ${BSTEPS:-30} --warmup 5 --no-cpu-baseline $BARGS > $O/tenv_${tag}_$c.json 2> $O/tenv_${tag}_$c.err || { tail -20 $O/tenv_${tag}_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/tenv_${tag}_$c.json'));r=d['roofline'];print('tune [$kv] $c',d['value'],d['ms_per_step'],r.get('launch_us'))" ;;
    bench*)
      c=${s#bench}; c=${c:-c3}
      timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])" ;;
  esac
done
