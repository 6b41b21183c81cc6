#!/bin/bash
# MFMA utilisation and HBM bytes of the C3 weight GEMMs: a kernel trace plus
# one rocprofv3 --pmc pass per counter group (kernel-trace only, no sys/runtime
# tracing), each under its own time limit; summarised by scripts/gemm_pmc_summarize.py.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_pmc
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i -E "mfma|GRBM_GUI_ACTIVE|SQ_BUSY_CYCLES" $O/avail.txt | head -40 > $O/avail_mfma.txt || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 $R/scripts/prof_gemm.py > $O/trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma -o mfma -- python3 $R/scripts/prof_gemm.py > $O/mfma.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 --kernel-trace --output-format csv -d $O/mops -o mops -- python3 $R/scripts/prof_gemm.py > $O/mops.log 2>&1 || echo "MOPS_I8 pass failed"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- python3 $R/scripts/prof_gemm.py > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- python3 $R/scripts/prof_gemm.py > $O/write.log 2>&1 || exit 1
cd $R && python3 scripts/gemm_pmc_summarize.py $O > $O/summary.json && cat $O/summary.json
