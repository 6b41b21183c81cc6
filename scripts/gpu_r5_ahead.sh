#!/bin/bash
# Round 5: C4 beam launch with two shared chunks in flight ahead
# (LLM_BEAM_AHEAD=2, tuning build as the product library for both arms),
# its stamps, and the kernel trace of the product C4 step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/ahead
mkdir -p $O /tmp/abt
cd $R
cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
for r in 1 2; do
  for a in 1 2; do
    LLM_BEAM_AHEAD=$a LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.ahead$a.$r.json 2> $O/c4.ahead$a.$r.err || { tail -5 $O/c4.ahead$a.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.ahead$a.$r.json'));print('c4 ahead $a round $r', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
  done
done
LLM_BEAM_AHEAD=2 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py --tag _ahead2 > $O/stamps_c4_ahead2.txt 2>&1 || { tail $O/stamps_c4_ahead2.txt; exit 1; }
grep -E "kernel span|first load|^exit|by seq" $O/stamps_c4_ahead2.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_graph -o tr -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --config c4 > $O/c4_graph.json 2> $O/c4_graph.err || { tail -5 $O/c4_graph.err; exit 1; }
cd $R && python3 scripts/analyze_trace.py $(ls $O/c4_graph/*/tr_kernel_trace.csv $O/c4_graph/tr_kernel_trace.csv 2>/dev/null | head -1) --by-grid > $O/step_timeline_c4.txt
head -4 $O/step_timeline_c4.txt
