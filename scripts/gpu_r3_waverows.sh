#!/bin/bash
# One-wave LayerNorm / quantiser launches (in-tree build) vs the 256-thread
# ones (ab_old/): parity tests, then a same-box A/B at C3 / C4 / C1.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/waverows
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py tests/test_c3_properties_gpu.py tests/test_c4_beams_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for c in ${CONFIGS:-c3 c4 c1}; do
    for v in old new; do
      if [ $v = old ]; then LP=$R/ab_old; else LP=; fi
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.$v.$r.json 2> $O/$c.$v.$r.err || { tail -5 $O/$c.$v.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$c.$v.$r.json'));print('$c $v $r', d['value'], d['ms_per_step'])"
    done
  done
done
