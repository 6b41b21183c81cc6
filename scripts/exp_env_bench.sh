#!/bin/bash
# GPU tests, then the C3 bench under each "VAR=value ..." setting given as an argument.
set -o pipefail
mkdir -p gpurun_out/eb
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/eb/tests.log 2>&1 || { tail -40 gpurun_out/eb/tests.log; exit 1; }
tail -1 gpurun_out/eb/tests.log
CFG=${CFG:-c3}
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/eb/b$i.json 2> gpurun_out/eb/b$i.err || { tail gpurun_out/eb/b$i.err; exit 1; }
  echo "[$envs] $(python -c "import json;d=json.load(open('gpurun_out/eb/b$i.json'));print(d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['roofline']['frac'])")"
done
