#!/bin/bash
# Fast iteration: selected GPU tests (TESTS, default: decoder + gemm + c3 props),
# then short benches of the configs in CONFIGS (default c2 c3 c4), no CPU baseline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
T=${TESTS:-tests/test_decoder_gpu.py tests/test_gemm_gpu.py tests/test_c3_properties_gpu.py}
timeout -k 10 900 python -u -m pytest $T -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit 1
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$c.json'));print('$c', d['value'], 'tok/s', d['ms_per_step'], 'ms', 'attn', d['roofline']['launch_us'], 'us')"
done
