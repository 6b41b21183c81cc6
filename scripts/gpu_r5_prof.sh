#!/bin/bash
# Round 5 profiles: C2's attention in the step vs alone (graph-mode kernel
# trace, then eager-mode PMC passes: bytes, L2 hits, waves), the C4 step's
# kernel trace (the beam launch in the step), per-wave stamps of the C4 beam
# launch by split / head / sequence / CU load, and the C3 strong-scaling
# per-GPU points (8 / 16 / 32 rows) with a trace of the 8-row step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/prof
mkdir -p $O
cd /tmp
B="python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline"
if [ -z "$SKIP_C2" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_graph -o tr -- $B --config c2 > $O/c2_graph.json 2> $O/c2_graph.err || { tail -5 $O/c2_graph.err; exit 1; }
  LLM_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2_eager -o tr -- $B --config c2 > /dev/null 2> $O/c2_eager.err || { tail -5 $O/c2_eager.err; exit 1; }
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    N=$(echo $P | cut -d' ' -f1)
    LLM_GRAPH=0 timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/c2_pmc_$N -o p -- $B --config c2 > /dev/null 2> $O/c2_pmc_$N.err || { tail -5 $O/c2_pmc_$N.err; exit 1; }
  done
  cd $R
  python3 scripts/instep_vs_alone.py $O/c2_graph > $O/c2_instep_vs_alone.txt
  echo "eager:" >> $O/c2_instep_vs_alone.txt
  python3 scripts/instep_vs_alone.py $O/c2_eager $O/c2_pmc_* >> $O/c2_instep_vs_alone.txt
  cat $O/c2_instep_vs_alone.txt
  python3 scripts/analyze_trace.py $(ls $O/c2_graph/*/tr_kernel_trace.csv $O/c2_graph/tr_kernel_trace.csv 2>/dev/null | head -1) --by-grid > $O/step_timeline_c2.txt
  cd /tmp
fi
if [ -z "$SKIP_C4" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_graph -o tr -- $B --config c4 > $O/c4_graph.json 2> $O/c4_graph.err || { tail -5 $O/c4_graph.err; exit 1; }
  cd $R
  python3 scripts/analyze_trace.py $(ls $O/c4_graph/*/tr_kernel_trace.csv $O/c4_graph/tr_kernel_trace.csv 2>/dev/null | head -1) --by-grid > $O/step_timeline_c4.txt
  head -12 $O/step_timeline_c4.txt
  mkdir -p /tmp/abt && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
  LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py --tag _il > $O/stamps_c4_il.txt 2>&1 || { tail $O/stamps_c4_il.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_c4_il.txt | grep -v "streaming per us"
  cd /tmp
fi
if [ -z "$SKIP_STRONG" ]; then
  cd $R && bash scripts/gpu_r5_strong.sh || exit 1
fi
