#!/bin/bash
# Wide Gram LDS-read ablations at configs[1] (tuning build, timing only): gram_diag 0 full, 128 no B
# reads in the loop, 256 no A reads, 384 neither, alternating with the full kernel.
#   bash tools/gpu_r6_wide_lds.sh TAG   -> gpurun_out/TAG_wide_lds.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"
for d in 0 128 256 384 0 128 384; do
  OB_GRAM_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py 2>/dev/null | tee -a gpurun_out/${1:-wl}_wide_lds.txt || exit 1
done
