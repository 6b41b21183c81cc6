#!/bin/bash
# 2-rank rehearsal of bench.py's N-GPU path on one GPU (gloo, ranks share
# cuda:0, outputs gathered through host memory): C2 and C3, logits and ids.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dist
mkdir -p $O
cd $R
for c in c2 c3; do
  for gth in ids logits; do
    LLM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config $c --steps 10 --warmup 3 \
      --no-cpu-baseline --gather $gth > $O/$c.$gth.json 2> $O/$c.$gth.err || { tail -20 $O/$c.$gth.err; exit 1; }
    tail -1 $O/$c.$gth.json | cut -c1-400
  done
done
