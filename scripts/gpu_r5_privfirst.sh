#!/bin/bash
# Round 5: C4's beam kernel with the beam-private chunks processed before the
# shared ones (tuning build, LLM_BEAM_PRIVFIRST=1): the C4-state oracle test
# through it, then same-box A/B against the product form.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/privfirst
mkdir -p $O /tmp/abt
cd $R
cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
LLM_BEAM_PRIVFIRST=1 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python -u -m pytest \
  "tests/test_decoder_long_context_gpu.py::test_int8_c4_beam_state_attention_vs_oracle" -m gpu -x -v -s \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $O/test.log 2>&1
rc=$?; grep -E "C4 state|passed|failed|FAILED|Error" $O/test.log | head -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for f in 0 1; do
    LLM_BEAM_PRIVFIRST=$f LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.pf$f.$r.json 2> $O/c4.pf$f.$r.err || { tail -5 $O/c4.pf$f.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.pf$f.$r.json'));r=d['roofline'];print('c4 privfirst $f round $r', d['value'], d['ms_per_step'], r['launch_us'])"
  done
done
echo done
