set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
for k in 2.5 3 3.5 4 5; do
  OB_MM_KAPPA=$k OB_MM_TRACE=1 timeout -k 10 200 python bench.py --mm --cpu-seconds 0 > gpurun_out/kap_$k.json 2> gpurun_out/kap_$k.err || exit 1
  echo "kappa $k: $(python3 -c "import json;print(json.load(open('gpurun_out/kap_$k.json'))['value'])") retries: $(grep -c 'round 0 at' gpurun_out/kap_$k.err) batches, $(grep 'round 0 at' gpurun_out/kap_$k.err | awk '{s+=$7} END {print s}') flagged fits, round2 $(grep -c 'round 1 at' gpurun_out/kap_$k.err)"
done
