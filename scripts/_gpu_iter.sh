set -o pipefail
mkdir -p gpurun_out/quick
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick/b_$name.json 2> gpurun_out/quick/b_$name.err || { tail gpurun_out/quick/b_$name.err; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/quick/b_$name.json'));print(d['value'], d['ms_per_step'], d['roofline']['launch_us'])")"
}
run mb1 LLM_MICROBATCHES=1
run pp1w2 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=1 LLM_MB_ATTN_WAVES=2
run pp1w3 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=1 LLM_MB_ATTN_WAVES=3
run pp1w4 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=1 LLM_MB_ATTN_WAVES=4
run pp1w6 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=1 LLM_MB_ATTN_WAVES=6
run pp0w4 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=0 LLM_MB_ATTN_WAVES=4
run pp0 LLM_MICROBATCHES=2 LLM_MB_PINGPONG=0
