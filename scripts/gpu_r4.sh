#!/bin/bash
# Round-4 session: GPU parity suite (new tests first), then bench lines
# (CONFIGS, default c3 c2) without the CPU baseline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|Error" gpurun_out/gpu_tests.log | head -30
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c3 c2}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])"
done
