#!/bin/bash
# Pieced resample (option rs_pieces): the bitwise tests, then timing at configs[1] (10k) and the
# 1,250 share for OB_RS_PIECES = 1, 2, 4 (tuning build), alternating.
#   bash tools/gpu_r6_pieces.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-pc}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "pieced or double_buffered or deterministic or segment_boundary" > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"
for r in $(seq ${PASSES:-2}); do
  for v in ${PIECES:-1 2 4}; do
    for R in ${SIZES:-10000 1250}; do
      out=gpurun_out/${T}_p${v}_${R}_$r.json
      OB_RS_PIECES=$v timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 \
        > $out 2> ${out%.json}.err || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('rs_pieces=$v $R',round(d['value']),round(d['ms_per_step'],3),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
