#!/bin/bash
# GEMM byte attribution: o_proj / mlp_fc2 forms (scripts/prof_gemm_forms.py)
# under a kernel trace, then one --pmc pass per counter (kernel-trace only);
# plus the production decode step's GEMM PMC (scripts/gpu_gemm_pmc.sh).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_attr
mkdir -p $O
cd /tmp
timeout -k 10 200 python3 $R/scripts/prof_gemm_forms.py > $O/plan.json 2> $O/plan.err || { tail $O/plan.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 $R/scripts/prof_gemm_forms.py > /dev/null 2> $O/trace.err || { tail $O/trace.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o f -- python3 $R/scripts/prof_gemm_forms.py > /dev/null 2> $O/fetch.err || { tail $O/fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o w -- python3 $R/scripts/prof_gemm_forms.py > /dev/null 2> $O/write.err || { tail $O/write.err; exit 1; }
cd $R && python3 scripts/gemm_attr_summarize.py $O $O/plan.json > $O/summary.json && python3 -c "
import json
for f in json.load(open('$O/summary.json'))['forms']:
    print(f['gemm'], 'NT%d w%d mr%d ks%d x%d' % (f['NT'], f['waves'], f['mrows'], f['kslices'], f['xcd_map']), f['us'], 'us fetch/model', f['fetch_pmc_over_model'], 'write/out', f['write_pmc_over_out'], 'pmc/unique', f['pmc_over_unique'])
"
bash $GRAFT_REPO_ROOT/scripts/gpu_gemm_pmc.sh > /dev/null || exit 1; cp $GRAFT_REPO_ROOT/gpurun_out/gemm_pmc/summary.json $GRAFT_REPO_ROOT/gpurun_out/gemm_attr/step_summary.json
