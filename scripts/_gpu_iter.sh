set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/quick/tests.log 2>&1 || { tail -60 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
