#!/bin/bash
# SQ counters of the level-1 kernel under the OB_L1_DIAG ablations (tools/l1_ablate.sh), one
# rocprofv3 pass per variant. usage: bash tools/pmc_l1.sh TAG "0 1 3"  -> gpurun_out/TAG_l1pmc_*.txt
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
TAG=${1:-rXX}
VARIANTS=${2:-"0 1 3 11 16 20"}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
for v in $VARIANTS; do
  OB_L1_DIAG=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/${TAG}_l1pmc_$v" -o run -- \
    python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_l1pmc_$v.log" 2>&1
  (cd "$REPO" && python tools/pmc_clock.py "$OUT/${TAG}_l1pmc_$v" ob_level1_kernel | tail -1 | sed "s/^/diag=$v /") \
    | tee -a "$OUT/${TAG}_l1pmc.txt"
done
