"""Per-kernel VGPR / spill / occupancy / LDS summary of a HIP source for gfx950.
    python scripts/kernel_resources.py pagedattention-.../csrc/gemm.hip"""
import re
import subprocess
import sys
from pathlib import Path

root = Path(__file__).resolve().parents[1]
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       f"-I{root / 'include'}",
       f"-I{root / 'pagedattention-based-transformer-decoder-inference-framework_amd' / 'csrc'}",
       "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
short = {"VGPRs": "vgpr", "AGPRs": "agpr", "VGPRs Spill": "spill", "ScratchSize [bytes/lane]": "scratch",
         "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds"}
for line in out.splitlines():
    m = re.search(r"(?:remark: |\s)(Function Name|VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|"
                  r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        if cur:
            print(cur)
        cur = v[:72]
    else:
        cur += f"  {short[k]}={v}"
print(cur)
