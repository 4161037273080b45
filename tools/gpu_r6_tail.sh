#!/bin/bash
# Tail stream (option tail_stream): its ordering / bitwise tests and the parity set under it, then
# timing at configs[1] (10k) and the 1,250 share, OB_TAIL_STREAM = 0 / 1 (tuning build), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-ts}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "tail_stream or pieced or double_buffered or deterministic or segment_boundary or device_api" \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"
OB_TAIL_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_gram_i8.py \
  -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests_on.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests_on.log; exit 1; }
echo "under OB_TAIL_STREAM=1: $(tail -1 gpurun_out/${T}_tests_on.log)"
for r in $(seq ${PASSES:-2}); do
  for v in 0 1; do
    for R in ${SIZES:-10000 1250}; do
      out=gpurun_out/${T}_t${v}_${R}_$r.json
      OB_TAIL_STREAM=$v timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 \
        > $out 2> ${out%.json}.err || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('tail_stream=$v $R',round(d['value']),round(d['ms_per_step'],3),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
