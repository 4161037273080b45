#!/bin/bash
# SQ / MFMA / memory counters of the Machado-Mata IPM passes (mm_assemble, mm_affine, mm_final) at
# configs[4] (bench.py --mm, one step), one rocprofv3 pass per counter group. On the GPU box:
#   bash tools/pmc_mm.sh TAG   -> gpurun_out/TAG_pmc_mm.txt
set -euo pipefail
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="GRBM_GUI_ACTIVE SQ_WAVES"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=1
for P in "$P1" "$P2" "$P3" "$P4"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/${TAG}_pmcm$i" -o run -- \
    python3 "$REPO/bench.py" --mm --steps 1 --warmup 0 --cpu-seconds 0 > "$OUT/${TAG}_pmcm$i.log" 2>&1
  i=$((i+1))
done
cd "$REPO"
for k in "mm_assemble_mfma_kernel<16, true>" "mm_affine_kernel<16>" "mm_final_kernel<16>"; do
  echo "## $k"
  for i in 1 2 3 4; do python tools/pmc_sum.py "$OUT/${TAG}_pmcm$i" "$k"; done
done > "$OUT/${TAG}_pmc_mm.txt"
cat "$OUT/${TAG}_pmc_mm.txt"
