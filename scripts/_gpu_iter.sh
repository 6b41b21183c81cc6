set -o pipefail
mkdir -p gpurun_out/quick
bash scripts/gpu_quick.sh "1 0" "2 0" || exit 1
LLM_MICROBATCHES=1 bash scripts/trace_step.sh it2
