set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/quick/tests.log 2>&1 || { tail -60 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick/b_c4.json 2> gpurun_out/quick/b_c4.err || { tail gpurun_out/quick/b_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/quick/b_c4.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
