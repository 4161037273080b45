#!/bin/bash
# Split wide Gram (gram_tile 3 / the engine's rule at small shares): the Gram bitwise test and the
# parity set, then timing at the driver's per-GPU shares, the in-tree library against the same
# library with the split forced off (OB_GRAM_TILE unset vs the rule without split via tuning build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-sp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram_i8.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/${T}_tests.log)"
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"
for r in 1 2; do
  for v in "" "OB_GRAM_TILE=1" "OB_GRAM_TILE=2"; do
    for R in ${SIZES:-1250 1000 10000}; do
      out=gpurun_out/${T}_$(echo "$v" | tr -dc '0-9')_${R}_$r.json
      env $v timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 > $out 2> ${out%.json}.err \
        || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('[$v] $R',round(d['value']),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
