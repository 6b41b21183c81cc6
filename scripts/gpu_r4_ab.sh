#!/bin/bash
# Same-box A/B of bench lines: VARIANTS (space-separated name=spec) x CONFIGS x ROUNDS.
# spec: "new" (in-tree product library), "old" (ab_old/libllm_decoder_hip.so),
# or "tune:ENV=VAL[,ENV=VAL]" (the tuning build copied to ab_tune/, with those switches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c4 c2 c3}; do
    for v in ${VARIANTS:-new=new old=old}; do
      name=${v%%=*}; spec=${v#*=}; LP=; ENVS=
      case $spec in
        old) LP=$R/ab_old ;;
        tune:*) LP=$R/ab_tune; ENVS=$(echo ${spec#tune:} | tr ',' ' ') ;;
      esac
      env $ENVS LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > $O/$c.$name.$r.json 2> $O/$c.$name.$r.err || { echo "bench $c $name failed"; tail -5 $O/$c.$name.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$c.$name.$r.json'));print('$c $name round $r', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
    done
  done
done
