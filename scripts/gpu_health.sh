#!/bin/bash
# Health round: smoke, then the C3 (default), C4 and C1 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print('c3',d['value'],d['ms_per_step'],d['roofline']['frac'])"
timeout -k 10 400 python bench.py --config c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -5 gpurun_out/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print('c4',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || { tail -5 gpurun_out/bench_c1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c1.json'));print('c1',d['value'],d['ms_per_step'])"
