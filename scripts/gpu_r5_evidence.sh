#!/bin/bash
# Round-5 evidence on the final head: step timelines + kernel stats (C3, C4,
# C2, C3 at 8 rows), PMC traffic of the decoder's own attention launch (C3,
# C4), and the per-GPU points of C3's strong curve (8 / 16 / 32 rows).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ev
mkdir -p $O
cd $R
for B in 8 16 32; do
  timeout -k 10 300 python bench.py --global-batch $B --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_rows$B.json 2> $O/bench_c3_rows$B.err || { tail -5 $O/bench_c3_rows$B.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c3_rows$B.json'));print('rows $B', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
done
for c in c3 c4 c2 c5 c3b8; do
  if [ $c = c3b8 ]; then args="--config c3 --global-batch 8"; else args="--config $c"; fi
  bash scripts/trace_step.sh r05f_$c $args || { echo "trace $c failed"; tail -5 gpurun_out/trace_r05f_$c/bench.err; exit 1; }
  f=$(find gpurun_out/trace_r05f_$c -name "*kernel_trace.csv" | head -1)
  python3 scripts/analyze_trace.py $f --by-grid > $O/step_timeline_$c.txt || exit 1
  cp $(find gpurun_out/trace_r05f_$c -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$c.csv
  head -4 $O/step_timeline_$c.txt
done
for c in c3 c4; do
  DEC=--decoder timeout -k 10 600 bash scripts/gpu_pmc.sh $c || { echo "pmc $c failed"; exit 1; }
  cp gpurun_out/pmc_attention_$c.json $O/
  python -c "import json;d=json.load(open('$O/pmc_attention_$c.json'));print('$c pmc', {k: d[k] for k in d if 'ratio' in k or 'over' in k})"
done
echo evidence done
