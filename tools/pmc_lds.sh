#!/bin/bash
# LDS counters of the resample kernels (bank conflicts, LDS issue stalls) in one rocprofv3 pass.
#   bash tools/pmc_lds.sh TAG   -> gpurun_out/TAG_pmc_lds_*.txt
set -euo pipefail
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/${TAG}_pmc_lds" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_pmc_lds.log" 2>&1
cd "$REPO"
for k in ob_level1_kernel ob_count_kernel; do
  python tools/pmc_clock.py "$OUT/${TAG}_pmc_lds" "$k" > "$OUT/${TAG}_pmc_lds_${k}.txt"
  tail -2 "$OUT/${TAG}_pmc_lds_${k}.txt"
done
