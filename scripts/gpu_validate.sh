#!/bin/bash
# Validation round on a fresh box: every -m gpu test, smoke, then the C3 / C4 / C1 / C2 bench lines.
set -o pipefail
bash scripts/gpu_tests.sh || exit 1
bash scripts/gpu_health.sh || exit 1
timeout -k 10 300 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -5 gpurun_out/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print('c2',d['value'],d['ms_per_step'])"
