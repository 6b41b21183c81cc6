#!/bin/bash
# Round-3 GPU session: parity tests (whole -m gpu suite), then the C3 bench
# line and C2 / C4 lines.  Outputs under gpurun_out/r3/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/log
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $O/$name.err; tail -40 $O/$name.out; case $rc in 124|134|137|139) exit 1;; esac; fi
  tail -3 $O/$name.out
}
[ "${SKIP_TESTS:-0}" = 1 ] || run tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread -rf
[ "${SKIP_BENCH:-0}" = 1 ] || run bench_c3 600 python bench.py --steps ${STEPS:-30} --warmup 5
for c in ${CONFIGS:-}; do
  run bench_$c 600 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline
done
echo session-done
