#!/bin/bash
# Kernel-trace profile of the Heckman bench (bench.py --heckman): bash tools/profile_heckman.sh TAG -> gpurun_out/TAG_hk_*
set -euo pipefail
TAG=${1:-rXX}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_hk_stats" -o run -- \
  python3 "$REPO/bench.py" --heckman --steps 2 --warmup 1 --cpu-seconds 0 > "$OUT/${TAG}_hk_stats.log" 2>&1
cd "$REPO"
cat "$OUT/${TAG}_hk_stats.log" | grep metric || true
find "$OUT/${TAG}_hk_stats" -name '*kernel_stats.csv' -exec cat {} \;
