set -o pipefail
mkdir -p gpurun_out/exp1
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/exp1/tests.log 2>&1 || { tail -40 gpurun_out/exp1/tests.log; exit 1; }
tail -2 gpurun_out/exp1/tests.log
for cfg in "1 1 1" "2 1 1" "2 0 1" "2 1 0" "1 1 0"; do
  set -- $cfg
  LLM_MICROBATCHES=$1 LLM_MB_PINGPONG=$2 LLM_GRAPH=$3 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/exp1/b_$1$2$3.json 2> gpurun_out/exp1/b_$1$2$3.err || { tail gpurun_out/exp1/b_$1$2$3.err; exit 1; }
  echo "mb=$1 pp=$2 graph=$3 $(python -c "import json;d=json.load(open('gpurun_out/exp1/b_$1$2$3.json'));print(d['value'], d['ms_per_step'], d['roofline']['launch_us'])")"
done
