#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "=== $1" >> gpurun_out/session.log; }
step tests
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -50 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
step bench
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step rocprof
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/prof -name "*stats*" | head
echo done
