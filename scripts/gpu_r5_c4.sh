#!/bin/bash
# Round 5, C4 beam attention: the beam-group parity tests, a same-box A/B of
# the product library against AB_DIR (ab_base/: the previous revision) on C4,
# and per-wave stamps of the shipped form and of round 4's form
# (LLM_BEAM_INTERLEAVE=0), both through the tuning build.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/c4
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_c4_beams_gpu.py tests/test_kv_cache_gpu.py \
    tests/test_decoder_long_context_gpu.py -k "c4 or beam or grouped or Beam" -m gpu -x -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
AB_DIR=${AB_DIR:-ab_base} CONFIGS=${CONFIGS:-c4} ROUNDS=${ROUNDS:-3} bash scripts/gpu_lib_ab.sh || exit 1
mkdir -p /tmp/abt && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py > $O/stamps_il.txt 2>&1 || { tail $O/stamps_il.txt; exit 1; }
LLM_BEAM_INTERLEAVE=0 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py > $O/stamps_contig.txt 2>&1 || { tail $O/stamps_contig.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_il.txt | head -14
grep -E "exit |first load|kernel span" $O/stamps_contig.txt
