set -o pipefail
# configs[4] throughput for phase-1 fit strides (OB_MM_FIT_STRIDE)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
for f in ${STRIDES:-2 4 8 16}; do
  OB_MM_FIT_STRIDE=$f OB_MM_TRACE=1 timeout -k 10 200 python bench.py --mm --cpu-seconds 0 > gpurun_out/fs_$f.json 2> gpurun_out/fs_$f.err || exit 1
  echo "stride $f: $(python3 -c "import json;print(json.load(open('gpurun_out/fs_$f.json'))['value'])") flagged $(grep 'round 0 at' gpurun_out/fs_$f.err | awk '{s+=$7} END {print s}') round2 $(grep -c 'round 1 at' gpurun_out/fs_$f.err) phase1 $(grep 'phase 1 done' gpurun_out/fs_$f.err | awk '{s+=$6; n++} END {print s/n}') ms"
done
