#!/bin/bash
# Machado-Mata replicates per step (one batch each) at configs[4]'s shape: bench.py --mm --reps R.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in ${SIZES:-12 32 64 125}; do
  timeout -k 10 400 python bench.py --mm --reps $R --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/mmb_$R.json 2> gpurun_out/mmb_$R.err || { tail -20 gpurun_out/mmb_$R.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/mmb_$R.json').read().strip().splitlines()[-1]);print($R,round(d['value'],2),round(d['ms_per_step'],1),d['roofline'].get('max_ipm_iterations'),d.get('check'))"
done
