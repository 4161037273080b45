#!/bin/bash
# Round 6: the default library's GPU parity set (rs_double's rule on), then the 2 x 2-grid wide Gram
# (liboaxaca_boot_grid.so, OB_OZ_W_GRID=1) through the Gram / parity tests and a timing A/B at
# configs[1] and 2,500 replicates (both on the wide kernel), base / grid alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-grid}
L=$PWD/oaxaca-blinder-rs_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_gram_i8.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_base_tests.log 2>&1 || { tail -40 gpurun_out/${T}_base_tests.log; exit 1; }
echo "base: $(tail -1 gpurun_out/${T}_base_tests.log)"
OB_LIB_PATH=$L/liboaxaca_boot_grid.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gram_i8.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_grid_tests.log 2>&1 || { tail -40 gpurun_out/${T}_grid_tests.log; exit 1; }
echo "grid: $(tail -1 gpurun_out/${T}_grid_tests.log)"
for r in 1 2 3; do
  for v in base grid; do
    if [ $v = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_grid.so"; fi
    for R in 10000 2500; do
      out=gpurun_out/${T}_${v}_${R}_$r.json
      env $E timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 > $out 2> ${out%.json}.err \
        || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('$v $R',round(d['value']),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
