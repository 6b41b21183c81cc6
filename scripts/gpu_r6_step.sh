set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_generate_free_run_gpu.py tests/test_decoder_gpu.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06/free_run_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06/free_run_tests.log
timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --copies 64 > gpurun_out/r06/tune_gemm_c3.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/tune_gemm.py --M 64 --hid 4096 --copies 16 > gpurun_out/r06/tune_gemm_c5.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c3 > gpurun_out/r06/bench_c3_base.json 2> gpurun_out/r06/bench_c3_base.err || exit 1
tail -c 600 gpurun_out/r06/bench_c3_base.json
exit $rc
