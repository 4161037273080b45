#!/bin/bash
# A subset of the GPU suite (pytest -k EXPR) then, optionally, the default bench line.
#   bash tools/gpu_quick.sh TAG 'k expression' [bench]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=$1; K=$2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "$K" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
if [ "$3" = bench ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
    || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]);print(round(d['value']),round(d['roofline']['frac'],3),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()});print({k:(round(v,3) if isinstance(v,float) else v) for k,v in d['end_to_end'].items() if k!='what'})"
fi
