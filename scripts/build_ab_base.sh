#!/bin/bash
# Build the product library of git revision REV (default HEAD) into ab_base/
# for same-box A/Bs against the working tree (scripts/gpu_lib_ab.sh AB_DIR=ab_base).
set -e
R=$(cd $(dirname $0)/.. && pwd)
REV=${1:-HEAD}
W=/tmp/ab_base_src
rm -rf $W && git -C $R worktree prune && git -C $R worktree add -f --detach $W $REV > /dev/null
make -s -j8 -C $W/pagedattention-based-transformer-decoder-inference-framework_amd libllm_decoder_hip.so
mkdir -p $R/ab_base && cp $W/pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip.so $R/ab_base/
git -C $R worktree remove --force $W
echo "ab_base/libllm_decoder_hip.so = $(git -C $R rev-parse --short $REV)"
