#!/bin/bash
# Round 5: C3's 8-row point (8 GPUs, strong scaling): the attention launch's
# split count (standalone pa_decode_tune, split + pa_merge_kernel, fixed pages
# per split (32 = the automatic 16 splits); variant 1 = the product kernel, 10 its
# loads-only form, 8 the 8 KiB-stage 4-waves-per-SIMD form) and the step's
# kernel timeline.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/b8
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/tune_attention.py --B 8 --variants 1 10 8 --pps 16 24 32 48 64 --rounds 5 > $O/attn_b8.txt 2>&1 || { tail -5 $O/attn_b8.txt; exit 1; }
grep variant $O/attn_b8.txt
bash scripts/trace_step.sh r05_c3b8 --global-batch 8 || { tail -5 gpurun_out/trace_r05_c3b8/bench.err; exit 1; }
f=$(find gpurun_out/trace_r05_c3b8 -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py $f --by-grid > $O/step_timeline_c3_b8.txt && head -14 $O/step_timeline_c3_b8.txt
