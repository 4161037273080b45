#!/bin/bash
# Is the i8 Gram bound by the power its operands cost? The same kernel with its B fragments zeroed in
# registers after the LDS reads (OB_GRAM_DIAG=16: same instructions, loads and barriers) against the
# shipped one: Gram time (tools/gram_ablate.py) and, per setting, one rocprofv3 pass for the clock
# and MFMA busy cycles. Run on the GPU box:  bash tools/gram_power_ablate.sh TAG
#   -> gpurun_out/TAG_power.txt
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
: > "$OUT/${TAG}_power.txt"
for d in 0 16 0 16; do
  OB_GRAM_DIAG=$d timeout -k 10 180 python tools/gram_ablate.py 2>/dev/null | tee -a "$OUT/${TAG}_power.txt"
done
cd /tmp && export TMPDIR=/tmp
for d in 0 16; do
  OB_GRAM_DIAG=$d timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d "$OUT/${TAG}_pw$d" -o run -- \
    python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_pw$d.log" 2>&1
done
cd "$REPO"
for d in 0 16; do echo "OB_GRAM_DIAG=$d: $(python tools/pmc_clock.py "$OUT/${TAG}_pw$d" oz_gram_kernel)"; done \
  | tee -a "$OUT/${TAG}_power.txt"
