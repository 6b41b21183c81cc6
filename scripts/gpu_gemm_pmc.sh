#!/bin/bash
# MFMA utilisation and HBM bytes of a config's weight GEMMs (CFG = c3 / c5 / c2):
# a kernel trace plus one rocprofv3 --pmc pass per counter group (kernel-trace
# only, no sys/runtime tracing), each under its own time limit; summarised by
# scripts/gemm_pmc_summarize.py into $O/summary.json.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${CFG:-c3}
O=$R/gpurun_out/gemm_pmc_$CFG
mkdir -p $O
cd /tmp
export PROF_CONFIG=$CFG
[ "$CFG" = c5 ] && export PROF_LAYERS=${PROF_LAYERS:-4}
MOPS=SQ_INSTS_VALU_MFMA_MOPS_I8
[ "$CFG" = c2 ] && MOPS=SQ_INSTS_VALU_MFMA_MOPS_F16
P="python3 $R/scripts/prof_gemm.py"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- $P > $O/trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma -o mfma -- $P > $O/mfma.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc $MOPS --kernel-trace --output-format csv -d $O/mops -o mops -- $P > $O/mops.log 2>&1 || echo "$MOPS pass failed"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- $P > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- $P > $O/write.log 2>&1 || exit 1
cd $R && python3 scripts/gemm_pmc_summarize.py $O $CFG > $O/summary.json && python3 -c "
import json; d=json.load(open('$O/summary.json'))
for k, g in d['gemms'].items(): print('$CFG', k, g['median_us'], 'us', g['weight_GBps'], 'GB/s', 'mfma', g['mfma_util_vs_peak'], g['mfma_busy_frac_from_cycles'], 'pmc/unique', g['attribution']['pmc_over_unique'])"
