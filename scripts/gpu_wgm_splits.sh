#!/bin/bash
# Split-count sweep of the workgroup-merge FP16 attention at C2: the product
# build (automatic split count) against the tuning build placed in ab_old/
# with LLM_WGM_SPLITS forced (and LLM_WG_MERGE=0: split + merge launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wgm_splits
mkdir -p $O
run() {  # name, LD path, env...
  local n=$1 lp=$2; shift 2
  env "$@" LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run auto.$r "" X=1 || exit 1
  for s in ${SPLITS:-3 4 6 8}; do run s$s.$r $R/ab_old LLM_WGM_SPLITS=$s || exit 1; done
  run merge.$r $R/ab_old LLM_WG_MERGE=0 || exit 1
done
