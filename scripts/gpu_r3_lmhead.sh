#!/bin/bash
# LM head decomposition (tuning build, LLM_LM_MODE: 1 no MFMA, 2 no x staging,
# 4 no E loads, 6 neither x nor E) at the C3 / C4 / C2 shapes, kernel trace.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lmh
mkdir -p $O
TL=$R/pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so
cd /tmp
for shape in 64,50257,2048 32,50257,2048 16,50257,768; do
  for mode in 0 1 2 4 6; do
    n=$(echo $shape | tr , _)_m$mode
    LLM_CAPI_LIB=$TL LLM_LM_MODE=$mode LM_SHAPE=$shape timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o t -- python3 $R/scripts/time_lm_head.py > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
    f=$(find $O/$n -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'lm_head_kernel' in r['Name']: print('$n', r['Name'][:40], 'avg_us', round(float(r['AverageNs'])/1e3,2), 'calls', r['Calls'])
"
  done
done
