#!/bin/bash
# Quick GPU iteration: gpu tests, then bench under each env setting given as
# arguments ("MB PP" pairs), no CPU baseline.
set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/quick/tests.log 2>&1 || { tail -40 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
for cfg in "$@"; do
  set -- $cfg
  LLM_MICROBATCHES=$1 LLM_MB_PINGPONG=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick/b_$1$2.json 2> gpurun_out/quick/b_$1$2.err || { tail gpurun_out/quick/b_$1$2.err; exit 1; }
  echo "mb=$1 pp=$2 $(python -c "import json;d=json.load(open('gpurun_out/quick/b_$1$2.json'));print(d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['roofline']['frac'])")"
done
