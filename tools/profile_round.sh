#!/bin/bash
# Round profile of the headline bench (run on the GPU box from the repo root):
#   bench JSON, rocprofv3 kernel-trace stats, FETCH_SIZE and WRITE_SIZE passes (separate, per
#   MI355X_MICROARCH.md), and a GRBM_GUI_ACTIVE + MFMA-busy pass for the effective clock.
# usage: [SKIP_BENCH=1] [KERNEL=oz_gram_w_kernel] bash tools/profile_round.sh TAG   -> gpurun_out/TAG_*
set -euo pipefail
TAG=${1:-rXX}
KERNEL=${KERNEL:-oz_gram_w_kernel}
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
REPO=$PWD
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py > "$OUT/${TAG}_bench.json"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_stats" -o run -- \
  python3 "$REPO/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${TAG}_fetch" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/${TAG}_write" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d "$OUT/${TAG}_clock" -o run -- \
  python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_clock.log" 2>&1
cd "$REPO"
python tools/pmc_summary.py "$OUT/${TAG}_fetch" "$OUT/${TAG}_write" 1000000 20 10000 "$OUT/${TAG}_pmc_gram.json" "$KERNEL"
python tools/pmc_clock.py "$OUT/${TAG}_clock" "$KERNEL" > "$OUT/${TAG}_clock_mfma.txt"
cat "$OUT/${TAG}_pmc_gram.json" "$OUT/${TAG}_clock_mfma.txt"
find "$OUT/${TAG}_stats" -name '*kernel_stats.csv' -exec cat {} \;
