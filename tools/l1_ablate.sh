#!/bin/bash
# Level-1 ablations at the bench shape (timing only, wrong counts): OB_L1_DIAG 0 full, 1 no random
# bits, 3 = 1 + one round only, 11 = 3 + no m1 stores, 16 return after the Knuth-Yao staging, 20 = 16
# without the staging. Prints level1_ms per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
for d in ${VARIANTS:-0 1 3 11 16 20}; do
  OB_L1_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py ${REPS:-10000} 2>/dev/null | sed "s/^/l1diag=$d /" | tee -a gpurun_out/${TAG:-la}_l1_ablate.txt || exit 1
done
