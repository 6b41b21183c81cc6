#!/bin/bash
# Round-5 GPU session: the -m gpu suite (TESTS: a subset), smoke(), the C3
# bench line as the driver runs it, the launcher's 2-rank gloo rehearsal
# (bench.py --gpus 2 with no external launcher, both ranks on cuda:0) and the
# refusal of --gpus 2 over RCCL on a 1-GPU box.  Every GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
O=gpurun_out/r05
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
  tail -2 $O/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err \
  || { tail -20 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3',d['value'],d['ms_per_step'],d['scaling'],d['roofline']['frac'],d['cpu_baseline']['value'])"
# the launcher: two ranks started by bench.py itself, gloo, both on cuda:0
LLM_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --config c2 --steps 10 --warmup 3 \
  --cpu-budget 5 > $O/bench_c2_gloo2.json 2> $O/bench_c2_gloo2.err \
  || { tail -20 $O/bench_c2_gloo2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2_gloo2.json'));print('c2 gloo x2',d['n_gpus'],d['value'],d['per_rank_ms_per_step'],d['weak_scaling']['value'])"
# --gpus 2 over RCCL on one GPU must fail loudly, before any collective
timeout -k 10 120 python3 bench.py --gpus 2 --config c2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_nccl2_on1.out 2> $O/bench_nccl2_on1.err
rc=$?
echo "nccl --gpus 2 on 1 GPU: rc=$rc"; grep -h "needs one GPU per rank" $O/bench_nccl2_on1.err | head -2
[ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] || exit 1
