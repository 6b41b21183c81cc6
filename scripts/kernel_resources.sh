#!/bin/bash
# Per-kernel VGPR / spill / occupancy / LDS summary of a HIP source for gfx950.
#   bash scripts/kernel_resources.sh csrc/gemm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$(dirname $0)/../include \
  -I$(dirname $0)/../pagedattention-based-transformer-decoder-inference-framework_amd/csrc \
  -c "$1" -o /tmp/_kr.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
cur = None
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|ScratchSize \[bytes/lane\]|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name":
        if cur: print(cur)
        cur = v[:70]
    else:
        cur += "  " + k.split()[0] + ("Spill" if "Spill" in k else "") + "=" + v
print(cur)
'
