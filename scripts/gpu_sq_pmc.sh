#!/bin/bash
# SQ issue/wait breakdown of the decode-attention launches (C3 plain split
# kernel and the C4 beam-group kernel, both from scripts/ab_attention_lib.py):
# two SQ-only PMC passes with kernel-trace, within the 8-SQ-slot limit, then a
# per-kernel summary (gpurun_out/sq_pmc_summary.json).  MFMA=1 runs the
# tuning build with the MFMA beam kernel instead (LLM_BEAM_MFMA=1).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
ENVS=""
if [ "${MFMA:-0}" = 1 ]; then
  export LLM_BEAM_MFMA=1 LLM_CAPI_LIB=$R/pagedattention-based-transformer-decoder-inference-framework_amd/libllm_decoder_hip_tune.so
fi
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq1 -o sq1 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/sq2 -o sq2 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
python3 - $O <<'PY'
import csv, glob, json, sys, collections
O = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for d in ("sq1", "sq2"):
    for f in glob.glob(f"{O}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "pa_split_kernel" in n or "pa_beam_mfma" in n:
                vals[n][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
out = {"source": "scripts/gpu_sq_pmc.sh (rocprofv3 --pmc, two SQ-only passes, kernel-trace) over scripts/ab_attention_lib.py; per-dispatch medians",
       "note": "SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles summed over waves; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES",
       "kernels": {}}
for n, cs in vals.items():
    k = {"kernel": n}
    for c, per in cs.items():
        v = sorted(per.values())
        k[c] = v[len(v) // 2]
    wc = k.get("SQ_WAVE_CYCLES", 0) or 1
    k["frac_active"] = round(k.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
    k["frac_wait_any"] = round(k.get("SQ_WAIT_ANY", 0) / wc, 3)
    k["frac_issue_stall"] = round(k.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
    k["frac_valu_active"] = round(k.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
    if k.get("SQ_LDS_IDX_ACTIVE"):
        k["lds_bank_conflict_per_active"] = round(k.get("SQ_LDS_BANK_CONFLICT", 0) / k["SQ_LDS_IDX_ACTIVE"], 3)
    out["kernels"][n[:80]] = k
json.dump(out, open(f"{O}/sq_pmc_summary.json", "w"), indent=1)
for n, k in out["kernels"].items():
    print(n, {x: k[x] for x in k if x.startswith("frac")})
PY
