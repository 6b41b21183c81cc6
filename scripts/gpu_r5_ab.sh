#!/bin/bash
# Round 5 A/B session: the parity tests of the round's new forms (TESTS), the
# C4 beam attention's interleaved splits against AB_DIR (ab_base/: the
# previous revision's product library), the C2 fused MLP against the two GEMM
# launches (LLM_MLP_FUSE, slice widths 2 / 4 / 8), same box, alternating, and
# per-wave stamps of the C4 launch (tuning build).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/ab
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_c4_beams_gpu.py tests/test_kv_cache_gpu.py tests/test_mlp_fused_gpu.py tests/test_decoder_long_context_gpu.py} \
    -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_C4" ]; then
  AB_DIR=${AB_DIR:-ab_base} CONFIGS=c4 ROUNDS=${ROUNDS:-2} bash scripts/gpu_lib_ab.sh || exit 1
fi
if [ -z "$SKIP_C2" ]; then
  for r in $(seq ${ROUNDS:-2}); do
    for v in 0 ${SLICES:-2 4 8}; do
      LLM_MLP_FUSE=$([ $v = 0 ] && echo 0 || echo 1) LLM_MLP_SLICE=$v timeout -k 10 300 python bench.py \
        --config c2 --steps 30 --warmup 5 --no-cpu-baseline > $O/c2.mlp$v.$r.json 2> $O/c2.mlp$v.$r.err \
        || { tail -5 $O/c2.mlp$v.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/c2.mlp$v.$r.json'));print('c2 mlp slice $v round $r', d['value'], d['ms_per_step'])"
    done
  done
fi
if [ -z "$SKIP_STAMPS" ]; then
  mkdir -p /tmp/abt && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
  LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py > $O/stamps_il.txt 2>&1 || { tail $O/stamps_il.txt; exit 1; }
  LLM_BEAM_INTERLEAVE=0 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py > $O/stamps_contig.txt 2>&1 || { tail $O/stamps_contig.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_il.txt | head -14
  grep -E "exit |first load|kernel span" $O/stamps_contig.txt
fi
