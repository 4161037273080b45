#!/bin/bash
# Round 5: where the SUB2 Gram's time goes -- SQ/clock/L2 counters (tools/pmc_gram.sh) and the
# DIAG ablations on the tuning build (no MFMAs, no sub-tile loads, zero B operands).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/pmc_gram.sh r5g > gpurun_out/r5g_pmc.log 2>&1 || { tail -20 gpurun_out/r5g_pmc.log; exit 1; }
cat gpurun_out/r5g_pmc_gram_sq.txt
export OB_LIB_PATH=$PWD/oaxaca-blinder-rs_amd/liboaxaca_boot_tuning.so
for d in 0 2 4 16 0; do
  OB_GRAM_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py || exit 1
done
