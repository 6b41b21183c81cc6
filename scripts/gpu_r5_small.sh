#!/bin/bash
# Round 5: C3's small per-GPU batches (the strong-scaling points): the
# LayerNorm prologue at <= 16 rows (this tree vs ab_base/), and the
# workgroup-merge form forced to 8 splits at 8 rows (tuning build,
# LLM_WGM_SPLITS=8) against the automatic 16-split split + merge form.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/small
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py -m gpu -x -v \
    -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for B in 8 16; do
  AB_DIR=ab_base CONFIGS=c3 ROUNDS=2 STEPS=20 EXTRA="--global-batch $B" bash scripts/gpu_lib_ab.sh | sed "s/^/rows $B: /" || exit 1
done
mkdir -p /tmp/abt && cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
for r in 1 2; do
  for f in 0 8; do
    LLM_WGM_SPLITS=$f LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --global-batch 8 --steps 20 --warmup 5 --no-cpu-baseline > $O/b8.wgm$f.$r.json 2> $O/b8.wgm$f.$r.err || { tail -5 $O/b8.wgm$f.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b8.wgm$f.$r.json'));r=d['roofline'];print('rows 8 wgm_splits $f round $r', d['value'], d['ms_per_step'], r['launch_us'], r['kernel'][:70])"
  done
done
