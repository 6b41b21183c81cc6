#!/bin/bash
# After the fused o_proj: the decoder's own C2 attention launch PMC (the
# workgroup-merge + o_proj kernel), then the C2 bench line with its CPU baseline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DEC=--decoder bash scripts/gpu_pmc.sh c2 || exit 1
cp gpurun_out/pmc_attention_c2.json profiles/pmc_attention_c2.json
timeout -k 10 600 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
