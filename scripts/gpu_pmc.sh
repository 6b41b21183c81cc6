#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per pass, kernel-trace only)
# over the production paged-attention launch at C3, summarised with the
# gfx950 FETCH_SIZE correction into profiles-ready JSON.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
CFG=${1:-c3}
DEC=${DEC:-}   # DEC=--decoder: the decoder's own launch (llm_decoder_run_attention)
cd /tmp
timeout -k 10 300 python3 $R/scripts/prof_attention.py --config $CFG --iters 10 $DEC > $O/att_algo_$CFG.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/att_trace_$CFG -o att -- python3 $R/scripts/prof_attention.py --config $CFG --iters 10 $DEC > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/att_fetch_$CFG -o fetch -- python3 $R/scripts/prof_attention.py --config $CFG --iters 10 $DEC > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/att_write_$CFG -o write -- python3 $R/scripts/prof_attention.py --config $CFG --iters 10 $DEC > /dev/null || exit 1
cd $R
python3 scripts/pmc_summarize.py --fetch $O/att_fetch_$CFG --write $O/att_write_$CFG --algo-json $O/att_algo_$CFG.json --out $O/pmc_attention_$CFG.json
