#!/bin/bash
# After the INT8 workgroup-merge change: the decoder's own attention launch PMC
# at C3 and C1, then the C3 step trace (bench under rocprofv3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for c in ${PMC_CONFIGS:-c3 c1}; do
  DEC=--decoder bash scripts/gpu_pmc.sh $c || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/pmc_attention_$c.json'));print('$c', d['traffic_over_algorithmic'], d.get('nsplit'), d.get('form'))"
done
CONFIGS=${TRACE_CONFIGS:-c3} bash scripts/gpu_r3_traces.sh
