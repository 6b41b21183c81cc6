#!/bin/bash
# Round-3 bench lines for every BASELINE config (CPU baseline included), one
# process each, under their own time limits; outputs gpurun_out/benches/.
set -o pipefail
O=gpurun_out/benches
mkdir -p $O
for c in ${CONFIGS:-c3 c1 c2 c4 c5}; do
  echo "=== $c"
  if [ $c = c3 ]; then args=""; else args="--config $c"; fi
  timeout -k 10 600 python bench.py $args --steps ${STEPS:-30} --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench $c rc=$rc"; tail -20 $O/bench_$c.err; exit 1; fi
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d.get('ms_per_step_median_hip_events'), d['roofline']['frac'], d['roofline'].get('traffic_over_algorithmic'), (d.get('cpu_baseline') or {}).get('value'))"
done
