set -o pipefail
# count-kernel ablations at the bench shape: 0 full, 32 no LDS atomics, 64 no Philox, 96 neither
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
for d in ${DIAGS:-0 32 64 96}; do
  OB_GRAM_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py 2>/dev/null | tee -a gpurun_out/${TAG:-ca}_count_ablate.txt || exit 1
done
