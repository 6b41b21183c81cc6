#!/bin/bash
# Round 5: C4's beam attention with 4 beam groups' splits per 16-wave
# workgroup (tuning build, LLM_BEAM_QUADS=4: the groups of a CU meet at every
# shared-chunk barrier) -- first the C4-state oracle test through it (uniform
# groups only: the form needs equal barrier sequences), then same-box A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/quads
mkdir -p $O /tmp/abt
cd $R
cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
LLM_BEAM_QUADS=4 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python -u -m pytest \
  "tests/test_decoder_long_context_gpu.py::test_int8_c4_beam_state_attention_vs_oracle" -m gpu -x -v -s \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $O/test.log 2>&1
rc=$?; grep -E "C4 state|passed|failed|FAILED|Error" $O/test.log | head -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in "0 1" "4 1" "4 0"; do
    set -- $f
    LLM_BEAM_QUADS=$1 LLM_BEAM_PRIO=$2 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.q$1p$2.$r.json 2> $O/c4.q$1p$2.$r.err || { tail -5 $O/c4.q$1p$2.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.q$1p$2.$r.json'));r=d['roofline'];print('c4 quads $1 prio $2 round $r', d['value'], d['ms_per_step'], r['launch_us'])"
  done
done
echo done
