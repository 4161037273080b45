#!/bin/bash
# Chunk-count A/B (OB_TARGET_CHUNKS builds liboaxaca_boot_c40/_c48.so against the in-tree 32) at the
# driver's per-GPU shares of configs[2] strong (10k / 5k / 2.5k / 1,250 replicates), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for r in 1 2; do
  for v in base ${LIBS:-c40 c48}; do
    if [ $v = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
    for R in ${SIZES:-10000 5000 2500 1250}; do
      out=gpurun_out/ch_${v}_${R}_$r.json
      env $E timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 > $out 2> ${out%.json}.err \
        || { tail -20 ${out%.json}.err; exit 1; }
      python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('$v $R',round(d['value']),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
    done
  done
done
