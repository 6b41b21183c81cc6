#!/bin/bash
# Round 5: the per-GPU points of C3's strong-scaling curve measured on one GPU
# (--global-batch B on 1 rank = the rows each of 64/B ranks holds), then a
# kernel trace of the 8-row step (the N = 8 point).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05/strong
mkdir -p $O
cd $GRAFT_REPO_ROOT
for B in ${ROWS:-8 16 32}; do
  timeout -k 10 300 python3 bench.py --global-batch $B --steps 20 --warmup 5 --no-cpu-baseline \
    > $O/c3_b$B.json 2> $O/c3_b$B.err || { tail -5 $O/c3_b$B.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c3_b$B.json'));print('B',$B,d['value'],d['ms_per_step'],d['roofline']['launch_us'],d['roofline']['frac'],d['roofline']['kernel'][:90])"
done
[ -n "$NO_TRACE" ] && exit 0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_b8 -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --global-batch 8 --steps 4 --warmup 2 --no-cpu-baseline \
  > $O/trace_b8.json 2> $O/trace_b8.err || { tail -5 $O/trace_b8.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/analyze_trace.py $(ls $O/trace_b8/*/tr_kernel_trace.csv $O/trace_b8/tr_kernel_trace.csv 2>/dev/null | head -1) --by-grid > $O/step_timeline_b8.txt
cat $O/step_timeline_b8.txt | head -30
