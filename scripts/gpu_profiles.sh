#!/bin/bash
# Round profile refresh: full GPU tests, C3 bench under rocprofv3 --stats,
# attention PMC traffic (c3, c4), GEMM MFMA / HBM PMC at C3, step timelines.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
[ "${SKIP_TESTS:-0}" = 1 ] || { timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }; tail -2 $O/gpu_tests.log; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c3_bench.json 2> $O/prof_c3.err || { tail -20 $O/prof_c3.err; exit 1; }
cd $R
bash scripts/gpu_pmc.sh c3 || exit 1
bash scripts/gpu_pmc.sh c4 || exit 1
bash scripts/gpu_gemm_pmc.sh || exit 1
bash scripts/gpu_traces.sh c3 c2 c4 || exit 1
echo profiles-done
