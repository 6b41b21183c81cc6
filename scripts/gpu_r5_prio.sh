#!/bin/bash
# Round 5: C4 beam launch with progress-ranked wave priority (LLM_BEAM_PRIO,
# tuning build as the product library for both arms), stamps, and the C2/C3
# attention timed back to back vs rotating over the layers.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/prio
mkdir -p $O /tmp/abt
cd $R
cp pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so /tmp/abt/libllm_decoder_hip.so
for r in 1 2; do
  for p in 0 1; do
    LLM_BEAM_PRIO=$p LD_LIBRARY_PATH=/tmp/abt timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/c4.prio$p.$r.json 2> $O/c4.prio$p.$r.err || { tail -5 $O/c4.prio$p.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4.prio$p.$r.json'));print('c4 prio $p round $r', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
  done
done
LLM_BEAM_PRIO=1 LD_LIBRARY_PATH=/tmp/abt timeout -k 10 200 python scripts/beam_stamps.py --tag _prio > $O/stamps_c4_prio.txt 2>&1 || { tail $O/stamps_c4_prio.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c4_prio.txt | grep -v "streaming per us" | head -20
for c in c2 c3; do
  timeout -k 10 300 python scripts/attn_rotate.py --config $c > $O/rotate_$c.txt 2>&1 || { tail -5 $O/rotate_$c.txt; exit 1; }
  grep -v amdgpu $O/rotate_$c.txt
done
