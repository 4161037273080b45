#!/bin/bash
# f64 VALU instruction counts of ob_probit_kernel at bench.py --heckman's shape (one rocprofv3 --pmc
# pass; 4 SQ counters) -> the JSON bench.py --heckman prices its roofline with. Run on the GPU box:
#   [OB_HK_ERFC=0] bash tools/pmc_probit.sh TAG   -> gpurun_out/TAG_pmc_probit.json
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
  --output-format csv -d "$OUT/${TAG}_pmcp" -o run -- \
  python3 "$REPO/bench.py" --heckman --steps 1 --warmup 0 --cpu-seconds 0 > "$OUT/${TAG}_pmcp.log" 2>&1
cd "$REPO"
python tools/pmc_f64.py "$OUT/${TAG}_pmcp" ob_probit_kernel "$OUT/${TAG}_pmc_probit.json" rows=1000000 preds=20 reps=2000 ks=4 \
  "erfc=${ERFC_LABEL:-npdf_ncdf}"
cat "$OUT/${TAG}_pmc_probit.json"
