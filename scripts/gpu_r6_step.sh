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
    ov*)  # ov<k>[_<config>]: bench line with LLM_OVERLAP=k (no CPU baseline), A/B
      k=${s#ov}; c=c3; case $k in *_*) c=${k#*_}; k=${k%%_*};; esac
      LLM_OVERLAP=$k timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/ov${k}_$c.json 2> $O/ov${k}_$c.err || { tail -20 $O/ov${k}_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/ov${k}_$c.json'));print('ov$k $c',d['value'],d['ms_per_step'],d.get('ms_per_step_median_hip_events'))" ;;
    trace*)  # trace<k>: kernel trace of the C3 bench with LLM_OVERLAP=k
      k=${s#trace}
      LLM_OVERLAP=$k bash scripts/trace_step.sh ov$k --config c3 || exit 1
      f=$(ls gpurun_out/trace_ov$k/*kernel_trace.csv | head -1)
      if [ "$k" = 0 ]; then python scripts/analyze_trace.py $f | head -14; else python scripts/overlap_timeline.py $f; fi ;;
    wgm*)  # wgm<P>_<NS>[_<config>]: bench line with LLM_WGM_PARTS=P LLM_WGM_NSPLIT=NS
      v=${s#wgm}; P=${v%%_*}; r=${v#*_}; NS=${r%%_*}; c=c2; case $r in *_*) c=${r#*_};; esac
      LLM_WGM_PARTS=$P LLM_WGM_NSPLIT=$NS timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/wgm${P}_${NS}_$c.json 2> $O/wgm${P}_${NS}_$c.err || { tail -20 $O/wgm${P}_${NS}_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/wgm${P}_${NS}_$c.json'));r=d['roofline'];print('wgm P=$P NS=$NS $c',d['value'],d['ms_per_step'],r.get('launch_us'),r.get('frac'))" ;;
    ab*)  # ab<config>: same-box A/B of ab_base/ (scripts/build_ab_base.sh) against the tree
      c=${s#ab}; STEPS=30 AB_DIR=ab_base CONFIGS=$c ROUNDS=${ROUNDS:-2} timeout -k 10 1000 bash scripts/gpu_lib_ab.sh || exit 1 ;;
    k2nt*)  # k2nt<NT>[_<config>]: bench line with LLM_FC2_K2_NT=NT (fc2 as two k slices at 64 rows)
      v=${s#k2nt}; k=${v%%_*}; c=c5; case $v in *_*) c=${v#*_};; esac
      LLM_FC2_K2_NT=$k timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/k2nt${k}_$c.json 2> $O/k2nt${k}_$c.err || { tail -20 $O/k2nt${k}_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/k2nt${k}_$c.json'));print('k2nt$k $c',d['value'],d['ms_per_step'])" ;;
    env:*)  # env:<VAR>=<v>:<config>: bench line under that variable (A/B)
      v=${s#env:}; kv=${v%%:*}; c=${v#*:}
      env $kv timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/env_$c.json 2> $O/env_$c.err || { tail -20 $O/env_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/env_$c.json'));print('$kv $c',d['value'],d['ms_per_step'])" ;;
    bench*)
      c=${s#bench}; c=${c:-c3}
      timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])" ;;
  esac
done
