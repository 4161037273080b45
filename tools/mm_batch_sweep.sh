#!/bin/bash
# configs[4] throughput against the Machado-Mata batch width (replicates per GPU per step; the
# batch holds them all when the state budget allows, OB_MM_STATE_GB). usage: TAG=x bash tools/mm_batch_sweep.sh "2 8 12"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in ${1:-2 8}; do
  timeout -k 10 400 python bench.py --mm --reps $r --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/${TAG:-mm}_mm_r$r.json 2> gpurun_out/${TAG:-mm}_mm_r$r.err || { tail -20 gpurun_out/${TAG:-mm}_mm_r$r.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG:-mm}_mm_r$r.json').read().strip().splitlines()[-1]);print('reps/step $r', round(d['value'],2), 'ms/step', round(d['ms_per_step'],1), d['check'])"
done
