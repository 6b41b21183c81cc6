#!/bin/bash
# Beam-group kernel experiment: beam parity tests, then C4 bench arms.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/beam4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_c4_beams_gpu.py tests/test_kv_cache_gpu.py tests/test_decoder_long_context_gpu.py tests/test_decoder_gpu.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf -k "beam or c4 or group" > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log
case $rc in 124|134|137|139) exit 1;; esac
arm() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', d['value'], d['ms_per_step'], r['launch_us'], r['kernel'][-60:])"
}
for rep in 1 2; do
  arm old$rep LLM_BEAM4=0 || exit 1
  arm new$rep LLM_BEAM4=1 || exit 1
  arm minw3_$rep LLM_BEAM4=1 LD_LIBRARY_PATH=$R/ab_old || exit 1
done
for ns in 8 12 16 24; do arm ns$ns LLM_BEAM4_SPLITS=$ns || exit 1; done
