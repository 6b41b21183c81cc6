#!/bin/bash
# Same-box A/B of an environment knob: bash scripts/gpu_ab.sh VAR "v1 v2" "c2 c4" [rounds]
set -o pipefail
VAR=$1; VALS=$2; CFGS=$3; ROUNDS=${4:-2}
O=gpurun_out/ab; mkdir -p $O
for r in $(seq $ROUNDS); do
  for c in $CFGS; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > $O/$c_$v.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
      python -c "import json;d=json.load(open('$O/$c_$v.json'));print('round $r $c $VAR=$v', d['value'], 'tok/s', d['ms_per_step'], 'ms')"
    done
  done
done
