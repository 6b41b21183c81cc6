set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/quick/tests.log 2>&1 || { tail -60 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
LLM_MICROBATCHES=1 bash scripts/trace_step.sh it6
python3 scripts/analyze_trace.py gpurun_out/trace_it6/tr_kernel_trace.csv
for i in 1 2; do
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick/b_c3.json 2> gpurun_out/quick/b_c3.err || { tail gpurun_out/quick/b_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/quick/b_c3.json'));print(d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
done
