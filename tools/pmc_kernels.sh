#!/bin/bash
# SQ issue/wait counters of the resample kernels (level 1, counts) in one rocprofv3 pass each, plus
# GRBM_GUI_ACTIVE for the clock. Run on the GPU box from the repo root:
#   bash tools/pmc_kernels.sh TAG   -> gpurun_out/TAG_pmc_*.txt
set -euo pipefail
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/${TAG}_pmc_sq" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_pmc_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv \
  -d "$OUT/${TAG}_pmc_clk" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_pmc_clk.log" 2>&1
cd "$REPO"
for k in ob_level1_kernel ob_count_kernel oz_gram; do
  { python tools/pmc_clock.py "$OUT/${TAG}_pmc_sq" "$k"; python tools/pmc_clock.py "$OUT/${TAG}_pmc_clk" "$k"; } \
    > "$OUT/${TAG}_pmc_${k}.txt"
  tail -3 "$OUT/${TAG}_pmc_${k}.txt"
done
