#!/bin/bash
# Round 5: C4 beam split count around the automatic 8 with the interleaved,
# prioritised form (tuning build, LLM_BEAM_NSPLIT), same box, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/bns
mkdir -p $O /tmp/abt
cd $R
cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
for r in 1 2; do
  for f in 0 6 7 10; do
    LLM_BEAM_NSPLIT=$f LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.ns$f.$r.json 2> $O/c4.ns$f.$r.err || { tail -5 $O/c4.ns$f.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.ns$f.$r.json'));r=d['roofline'];print('c4 beam_nsplit $f round $r', d['value'], d['ms_per_step'], r['launch_us'])"
  done
done
echo done
