#!/bin/bash
# Phase-2 start offset sweep (OB_MM_DELTA2 scales the centred start's z/w offset): configs[4]
# throughput and the phase-2 iteration trace per setting. Run on the GPU box:
#   bash tools/mm_delta_sweep.sh TAG 1 0.3 0.1 ...   -> gpurun_out/TAG_delta.txt
set -o pipefail
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
TAG=$1; shift
mkdir -p gpurun_out
: > gpurun_out/${TAG}_delta.txt
for d in "$@"; do
  env OB_MM_TRACE=1 "${VAR:-OB_MM_DELTA2}=$d" timeout -k 10 240 python bench.py --mm --steps 2 --warmup 1 --cpu-seconds 0 --no-e2e \
    > gpurun_out/${TAG}_d$d.json 2> gpurun_out/${TAG}_d$d.err || { tail -20 gpurun_out/${TAG}_d$d.err; exit 1; }
  v=$(python -c "import json;print(round(json.loads(open('gpurun_out/${TAG}_d$d.json').read().strip().splitlines()[-1])['value'],2))")
  it=$(grep -c "iteration" gpurun_out/${TAG}_d$d.err)
  echo "${VAR:-OB_MM_DELTA2}=$d value=$v rep/s; $(grep 'after' gpurun_out/${TAG}_d$d.err | tail -3 | tr '\n' ' ')" | tee -a gpurun_out/${TAG}_delta.txt
  grep "round 0\|round 1" gpurun_out/${TAG}_d$d.err | tail -2 >> gpurun_out/${TAG}_delta.txt
done
