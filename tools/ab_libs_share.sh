#!/bin/bash
# Timing A/B of alternative builds at configs[1] (10k replicates) and at configs[2]'s per-GPU share
# (1,250): the in-tree library ("base") and liboaxaca_boot_NAME.so per NAME, base again last.
# usage: TAG=x bash tools/ab_libs_share.sh NAME...   -> gpurun_out/TAG_abs_*.json, summary on stdout
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for v in base "$@" base; do
  if [ "$v" = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
  for R in 10000 1250; do
    env $E timeout -k 10 300 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 \
      > gpurun_out/${TAG:-ab}_abs_${v}_$R.json 2> gpurun_out/${TAG:-ab}_abs_${v}_$R.err || { tail -20 gpurun_out/${TAG:-ab}_abs_${v}_$R.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${TAG:-ab}_abs_${v}_$R.json').read().strip().splitlines()[-1]);print('$v $R',round(d['value']),{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
  done
done
