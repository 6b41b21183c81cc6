#!/bin/bash
# One GPU session: parity tests, smoke, the default bench line, the other
# BASELINE configs, and a 2-rank gloo rehearsal of the multi-rank bench loop
# (ragged strong scaling, ids gather).  Outputs under gpurun_out/session/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/session
mkdir -p $O
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/log
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 $O/$name.err; tail -30 $O/$name.out; exit 1; fi
  tail -2 $O/$name.out
}
[ "${SKIP_TESTS:-0}" = 1 ] || run tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c3 600 python bench.py
for c in ${CONFIGS:-c1 c2 c4}; do
  run bench_$c 600 python bench.py --config $c --steps 20 --warmup 5
done
[ "${SKIP_DIST:-0}" = 1 ] || run dist_gloo 600 env LLM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --config c2 --global-batch 15 --gather ids --no-cpu-baseline
echo session-done
