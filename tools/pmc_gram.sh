#!/bin/bash
# SQ stall / LDS / L2 counters of the i8 Gram (oz_gram_kernel) at configs[1], one rocprofv3 pass per
# counter group (MI355X_MICROARCH.md: at most 8 SQ, 4 TCC counters a pass). Run on the GPU box:
#   bash tools/pmc_gram.sh TAG [KERNEL]   -> gpurun_out/TAG_pmc_gram_*.txt
set -euo pipefail
TAG=${1:-rXX}
K=${2:-oz_gram_kernel}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA"
P3="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/${TAG}_pmcg$i" -o run -- \
    python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_pmcg$i.log" 2>&1
  i=$((i+1))
done
cd "$REPO"
for i in 1 2 3; do python tools/pmc_clock.py "$OUT/${TAG}_pmcg$i" "$K"; done > "$OUT/${TAG}_pmc_gram_sq.txt"
cat "$OUT/${TAG}_pmc_gram_sq.txt"
