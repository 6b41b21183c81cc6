#!/bin/bash
# Round 5: pa_merge_kernel loading every split's (m, l) and first 16 partials
# in one round trip (and pa_merge_row_kernel through the same per-head
# helper) against ab_base/ (HEAD before the change): attention / decoder
# tests, then same-box A/B at C3's 8-row strong-scaling point and C4, then
# the M = 8 / 16 split-K sweep of the o_proj / fc2 GEMMs (tuning build).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/merge
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_pa_decode_gpu.py tests/test_c4_beams_gpu.py tests/test_decoder_gpu.py tests/test_decoder_long_context_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch 8" bash scripts/gpu_lib_ab.sh | sed "s/^/rows 8: /" || exit 1
AB_DIR=ab_base CONFIGS=c4 ROUNDS=2 bash scripts/gpu_lib_ab.sh || exit 1
for M in 8 16; do
  timeout -k 10 300 python scripts/tune_gemm_sk.py --M $M --reps 30 > $O/gemm_sk_M$M.txt 2>&1 || { tail -5 $O/gemm_sk_M$M.txt; exit 1; }
done
timeout -k 10 300 python scripts/tune_gemm.py --M 8 --reps 30 > $O/gemm_M8.txt 2>&1 || { tail -5 $O/gemm_M8.txt; exit 1; }
echo done1
# C4 beam split count with the interleaved + prioritised form (tuning build,
# LLM_BEAM_NSPLIT; 0 = the automatic 8): more splits than resident slots let
# early-finishing CUs take a second round
mkdir -p /tmp/abt && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
for r in 1 2; do
  for f in 0 12 16; do
    LLM_BEAM_NSPLIT=$f LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.ns$f.$r.json 2> $O/c4.ns$f.$r.err || { tail -5 $O/c4.ns$f.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.ns$f.$r.json'));r=d['roofline'];print('c4 beam_nsplit $f round $r', d['value'], d['ms_per_step'], r['launch_us'])"
  done
done
echo done2
