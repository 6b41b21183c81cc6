#!/bin/bash
# LM head with x staged once (<= 16 rows): parity tests, kernel times at the
# C2 shape and a 16-row K 2048 shape, then a C2 / C1 same-box A/B (ab_old/).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lmx1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for shape in 16,50257,768 16,50257,2048; do
  for v in old new; do
    if [ $v = old ]; then LP=$R/ab_old; else LP=; fi
    n=$(echo $shape | tr , _)_$v
    LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} LLM_CAPI_LIB=${LP:-$R/pagedattention-based-transformer-decoder-inference-framework_amd}/libllm_decoder_hip.so LM_SHAPE=$shape timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o t -- python3 $R/scripts/time_lm_head.py > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
    f=$(find $O/$n -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lm_head' in r['Name']: print('$n', r['Name'][:40], 'avg_us', round(float(r['AverageNs'])/1e3,2), [l for l in open('$O/$n.log').read().split(chr(10)) if 'max_abs' in l])
"
  done
done
cd $R
CONFIGS="c2 c1" ROUNDS=2 STEPS=30 bash scripts/gpu_lib_ab.sh
