#!/bin/bash
# Round-5 record session: the whole -m gpu suite, smoke(), then one full
# bench.py line per config (with the CPU baseline) into gpurun_out/r05_bench_<c>.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
  tail -2 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
for c in ${CONFIGS:-c3 c4 c2 c1 c5}; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r05_bench_$c.json 2> gpurun_out/r05_bench_$c.err \
    || { tail -20 gpurun_out/r05_bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'])"
done
# the N-rank strong path with the real decoder: C3's 64 rows over 2 and 4
# gloo ranks sharing this one GPU (bench.py starts the ranks itself; the
# timing is not a scaling number, the ranks share one device)
if [ -n "$GLOO_REHEARSAL" ]; then
  for n in 2 4; do
    LLM_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline --no-weak-extra > gpurun_out/r05_bench_c3_gloo$n.json 2> gpurun_out/r05_bench_c3_gloo$n.err \
      || { tail -20 gpurun_out/r05_bench_c3_gloo$n.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r05_bench_c3_gloo$n.json'));print('c3 gloo', d['n_gpus'], d['scaling'], d['config']['batch_per_gpu'], d['per_rank_ms_per_step'], d['process_group'], d['gather'])"
  done
fi
