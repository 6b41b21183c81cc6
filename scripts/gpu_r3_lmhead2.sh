#!/bin/bash
# LM head forms (tuning build, LLM_LM_FORM 0: 16 waves x 1 vocabulary tile,
# 1: 8 waves x 2 tiles) at the C3 / C4 / C2 shapes, kernel trace; then the
# product LM head parity tests.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lmh2
mkdir -p $O
TL=$R/pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so
cd /tmp
for shape in 64,50257,2048 32,50257,2048 16,50257,768; do
  for form in 0 1; do
    for mode in ${MODES:-0}; do
      n=$(echo $shape | tr , _)_f${form}_m$mode
      LLM_CAPI_LIB=$TL LLM_LM_FORM=$form LLM_LM_MODE=$mode LM_SHAPE=$shape timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o t -- python3 $R/scripts/time_lm_head.py > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
      f=$(find $O/$n -name "*kernel_stats.csv" | head -1)
      python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lm_head_kernel' in r['Name']: print('$n', r['Name'][:44], 'avg_us', round(float(r['AverageNs'])/1e3,2), 'calls', r['Calls'], open('$O/$n.log').read().strip().split(chr(10))[-1])
"
    done
  done
done
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "lm_head or argmax" -m gpu 2>&1 | tail -3
