#!/bin/bash
# configs[4] at a given batch width: kernel-trace stats (rocprofv3) and the phase trace (OB_MM_TRACE=1).
# usage: bash tools/mm_profile.sh TAG REPS  -> gpurun_out/TAG_mmstats/, TAG_mmtrace.log
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
TAG=${1:-mm}; R=${2:-12}
OUT=$PWD/gpurun_out; REPO=$PWD
mkdir -p "$OUT"
OB_MM_TRACE=1 timeout -k 10 300 python bench.py --mm --reps $R --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/${TAG}_mmtrace.json" 2> "$OUT/${TAG}_mmtrace.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_mmstats" -o run -- \
  python3 "$REPO/bench.py" --mm --reps $R --steps 1 --warmup 1 --cpu-seconds 0 > "$OUT/${TAG}_mmstats.log" 2>&1
find "$OUT/${TAG}_mmstats" -name '*kernel_stats.csv' -exec head -14 {} \; | cut -c1-160
grep "\[mm\]" "$OUT/${TAG}_mmtrace.log" | tail -30
