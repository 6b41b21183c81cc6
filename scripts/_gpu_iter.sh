set -o pipefail
bash scripts/gpu_round.sh && bash scripts/gpu_pmc.sh c3 && bash scripts/trace_step.sh c3 && python3 scripts/analyze_trace.py gpurun_out/trace_c3/tr_kernel_trace.csv > gpurun_out/trace_c3/analysis.txt && cat gpurun_out/pmc_attention_c3.json | head -30
