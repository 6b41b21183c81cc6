set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/quick/tests.log 2>&1 || { tail -40 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
for c in c3 c4 c2; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick/b_$c.json 2> gpurun_out/quick/b_$c.err || { tail gpurun_out/quick/b_$c.err; exit 1; }
  cat gpurun_out/quick/b_$c.json
done
