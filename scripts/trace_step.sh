#!/bin/bash
# Kernel-trace one bench configuration (env passed through) for timeline analysis.
#   bash scripts/trace_step.sh NAME [extra bench.py args]   (env: LLM_GRAPH=0 for eager launches)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NAME=$1
shift
mkdir -p $R/gpurun_out/trace_$NAME
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$NAME -o tr -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > $R/gpurun_out/trace_$NAME/bench.json 2> $R/gpurun_out/trace_$NAME/bench.err
