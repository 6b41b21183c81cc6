set -o pipefail
mkdir -p gpurun_out/quick
LLM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config c2 --steps 10 --warmup 3 > gpurun_out/quick/dist2_c2.json 2> gpurun_out/quick/dist2_c2.err || { tail -30 gpurun_out/quick/dist2_c2.err; exit 1; }
cat gpurun_out/quick/dist2_c2.json
