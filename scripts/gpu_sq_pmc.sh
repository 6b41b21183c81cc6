#!/bin/bash
# SQ issue/wait breakdown of the decode-attention launches (C3 plain split
# kernel and the C4 beam-group kernel, both from scripts/ab_attention_lib.py):
# two SQ-only PMC passes with kernel-trace, within the 8-SQ-slot limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq1 -o sq1 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/sq2 -o sq2 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
