#!/bin/bash
# Double-buffered resample (option rs_double): its bitwise test, then timing A/B against one buffer
# at configs[1] (10k) and configs[2]'s share (1,250), alternating, through the tuning build (OB_RS_DOUBLE).
#   bash tools/gpu_r6_rsdouble.sh TAG   -> gpurun_out/TAG_*.json, summary on stdout
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-rsd}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "double_buffered or deterministic or segment_boundary or device_api" > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"
for r in $(seq ${PASSES:-3}); do
  for v in 0 1; do
    for R in ${SIZES:-10000 1250}; do
      out=gpurun_out/${T}_d${v}_${R}_$r.json
      OB_RS_DOUBLE=$v timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 \
        > $out 2> ${out%.json}.err || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('rs_double=$v $R',round(d['value']),round(d['ms_per_step'],3),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
