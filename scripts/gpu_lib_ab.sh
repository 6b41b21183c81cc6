#!/bin/bash
# Same-box A/B of two product library builds through bench.py: the build in
# AB_DIR (default ab_old/; scripts/build_ab_base.sh makes ab_base/ from a git
# revision) via LD_LIBRARY_PATH, which the pybind module's RUNPATH yields to,
# against the in-tree build, alternating, CONFIGS (default c2 c4) x ROUNDS.
# EXTRA: more bench.py arguments (e.g. --global-batch 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lib_ab
AB=${AB_DIR:-ab_old}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c2 c4}; do
    for v in ${ORDER:-old new}; do
      if [ $v = old ]; then LP=$R/$AB; else LP=; fi
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline $EXTRA > $O/$c.$v.$r.json 2> $O/$c.$v.$r.err || { tail -5 $O/$c.$v.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$c.$v.$r.json'));r=d['roofline'];print('$c $v round $r', d['value'], d['ms_per_step'], r['launch_us'] if r else '')"
    done
  done
done
