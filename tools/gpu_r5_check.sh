#!/bin/bash
# Round 5 check on one box: the GPU suite, the default bench (driver form) and configs[2]'s
# per-GPU share. usage: bash tools/gpu_r5_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-r5c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${T}_gputests.txt 2>&1 || { tail -40 gpurun_out/${T}_gputests.txt; exit 1; }
tail -1 gpurun_out/${T}_gputests.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]);print(round(d['value']),round(d['roofline']['frac'],3),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()}, d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --reps 1250 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e \
  > gpurun_out/${T}_share1250.json 2> gpurun_out/${T}_share1250.err || { tail -30 gpurun_out/${T}_share1250.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_share1250.json').read().strip().splitlines()[-1]);print('share1250',round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
