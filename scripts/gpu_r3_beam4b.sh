#!/bin/bash
# Beam-group kernel arms, kernel-traced: split and merge times separately.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/beam4b
mkdir -p $O
export TMPDIR=/tmp
arm() {  # name env...
  local n=$1; shift
  cd /tmp
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o tr -- python3 $R/scripts/prof_attention.py --config c4 --iters 20 --decoder > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  cd $R
  echo "$n $(cat $O/$n.json)"
  f=$(find $O/$n -name "*kernel_stats.csv" | head -1)
  grep -E "pa_split|pa_beam|pa_merge" $f | awk -F'","' '{printf "   %s calls=%s avg_us=%.2f\n", substr($1,1,60), $2, $4/1000}'
}
arm old LLM_BEAM4=0 || exit 1
arm u1ns8 LLM_BEAM4=1 LLM_BEAM4_SPLITS=8 || exit 1
arm u1ns16 LLM_BEAM4=1 LLM_BEAM4_SPLITS=16 || exit 1
arm u2ns8 LLM_BEAM4=1 LLM_BEAM4_SPLITS=8 LD_LIBRARY_PATH=$R/ab_old || exit 1
arm u2ns16 LLM_BEAM4=1 LLM_BEAM4_SPLITS=16 LD_LIBRARY_PATH=$R/ab_old || exit 1
arm u2ns12 LLM_BEAM4=1 LLM_BEAM4_SPLITS=12 LD_LIBRARY_PATH=$R/ab_old || exit 1
