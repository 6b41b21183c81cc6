#!/bin/bash
# Quantising o_proj prologue + INT8 workgroup-merge attention: decoder parity
# tests, then a same-box A/B against the previous build (ab_old/) at C3 / C1 / C5.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/qpro
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py tests/test_c3_properties_gpu.py \
  tests/test_dist_gpu.py tests/test_pa_decode_gpu.py tests/test_gemm_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for c in ${CONFIGS:-c3 c1 c5}; do
    for v in old new; do
      if [ $v = old ]; then LP=$R/ab_old; else LP=; fi
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.$v.$r.json 2> $O/$c.$v.$r.err || { tail -5 $O/$c.$v.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$c.$v.$r.json'));r=d['roofline'];print('$c $v $r', d['value'], d['ms_per_step'], r['frac'], r['launch_us'], r['kernel'][:100])"
    done
  done
done
