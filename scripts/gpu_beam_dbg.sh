# Kernel-level timing of the beam-group attention forms (rocprofv3 kernel trace;
# host-side launch overhead excluded): MFMA full / load-only / compute-only,
# and the VALU BEAM form.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/pagedattention-based-transformer-decoder-inference-framework_amd
O=$R/gpurun_out/beam_dbg
mkdir -p $O
cd /tmp
for v in "mfma 0 1" "loadonly 1 1" "computeonly 2 1" "valu 0 0"; do
  set -- $v
  LLM_BEAM_MFMA_DBG=$2 LLM_BEAM_MFMA=$3 LLM_CAPI_LIB=$P/libllm_decoder_hip_tune.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o $1 -- python3 $R/scripts/ab_attention_lib.py > $O/$1.log 2>&1 || exit 1
  python3 - $O/$1 $1 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "beam" in n or "split_kernel<128, 16, false, 8192" in n or "merge_row" in n:
        print(sys.argv[2], n[:60], "avg us", round(float(r["AverageNs"]) / 1e3, 2), "calls", r["Calls"])
PY
done
