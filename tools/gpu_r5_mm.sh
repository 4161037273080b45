#!/bin/bash
# Machado-Mata at configs[4] on one box: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE passes
# (separate runs, MI355X_MICROARCH.md) over one bench step, summarised per kernel by
# tools/pmc_mm_traffic.py into gpurun_out/TAG_pmc_mm.json. usage: bash tools/gpu_r5_mm.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-r05mm}
OUT=$PWD/gpurun_out
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${T}_mmstats" -o run -- \
  python3 "$REPO/bench.py" --mm --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/${T}_mmstats.log" 2>&1 || { tail -20 "$OUT/${T}_mmstats.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/${T}_mm_$c" -o run -- \
    python3 "$REPO/bench.py" --mm --steps 1 --warmup 0 --cpu-seconds 0 > "$OUT/${T}_mm_$c.log" 2>&1 || { tail -20 "$OUT/${T}_mm_$c.log"; exit 1; }
done
cd "$REPO"
python tools/pmc_mm_traffic.py "$OUT/${T}_mm_FETCH_SIZE" "$OUT/${T}_mm_WRITE_SIZE" "$OUT/${T}_mm_FETCH_SIZE.log" > "$OUT/${T}_pmc_mm.json"
cat "$OUT/${T}_pmc_mm.json"
find "$OUT/${T}_mmstats" -name '*kernel_stats.csv' -exec head -16 {} \; | cut -c1-170
