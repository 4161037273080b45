#!/bin/bash
# Timing A/B of alternative builds (tools/build_alt.sh ... NAME): the in-tree library ("base") and
# oaxaca-blinder-rs_amd/liboaxaca_boot_NAME.so for each NAME, one short bench each, base again last.
# usage: TAG=x bash tools/ab_libs.sh NAME...   -> gpurun_out/TAG_ab_NAME.json, summary on stdout
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for v in base "$@" base; do
  if [ "$v" = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
  env $E timeout -k 10 300 python bench.py --cpu-seconds 0 --no-e2e --steps 10 --warmup 3 \
    > gpurun_out/${TAG:-ab}_ab_$v.json 2> gpurun_out/${TAG:-ab}_ab_$v.err || { tail -20 gpurun_out/${TAG:-ab}_ab_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG:-ab}_ab_$v.json').read().strip().splitlines()[-1]);print('$v',round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
