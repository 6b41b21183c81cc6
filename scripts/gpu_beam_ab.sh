#!/bin/bash
# A/B of the beam-group attention forms on one box: the MFMA kernel (product
# library) and the VALU BEAM form (tuning library, LLM_BEAM_MFMA=0), with a
# fixed-pages-per-split sweep, then the SQ counters of the MFMA form.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/beam_ab
mkdir -p $O
P=$R/pagedattention-based-transformer-decoder-inference-framework_amd
export AB_C4_PPS=${AB_C4_PPS:-16,32,64,128}
timeout -k 10 120 python3 $R/scripts/ab_attention_lib.py | tee $O/mfma.json || exit 1
LLM_BEAM_MFMA=0 LLM_CAPI_LIB=$P/libllm_decoder_hip_tune.so timeout -k 10 120 python3 $R/scripts/ab_attention_lib.py | tee $O/valu.json || exit 1
[ -n "$NO_PMC" ] && exit 0
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq1 -o sq1 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq2 -o sq2 -- python3 $R/scripts/ab_attention_lib.py > /dev/null || exit 1
python3 - <<PY
import csv, glob, collections
for d in ("sq1", "sq2"):
    for f in glob.glob("$O/%s/**/*counter_collection.csv" % d, recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "beam_mfma" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k, v in sorted(acc.items()):
            vals = list(v.values())
            print(d, k, "per dispatch avg", sum(vals) / len(vals))
PY
