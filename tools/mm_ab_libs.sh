#!/bin/bash
# Machado-Mata A/B of alternative builds (tools/build_alt.sh ob_mm.hip ... NAME), alternating
# base, NAME... for $PAIRS rounds so drift shows as spread, not as a difference.
# usage: PAIRS=3 TAG=x bash tools/mm_ab_libs.sh NAME...   -> gpurun_out/TAG_mmab.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for p in $(seq 1 ${PAIRS:-3}); do
  for v in base "$@"; do
    if [ "$v" = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
    env $E timeout -k 10 300 python bench.py --mm --steps 3 --warmup 1 --cpu-seconds 0 \
      > gpurun_out/${TAG:-mm}_mmab_$v.json 2> gpurun_out/${TAG:-mm}_mmab_$v.err || { tail -20 gpurun_out/${TAG:-mm}_mmab_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${TAG:-mm}_mmab_$v.json').read().strip().splitlines()[-1]);print('pair $p $v',round(d['value'],2),round(d['roofline']['assemble_ms'],1),d['roofline']['max_ipm_iterations'])" | tee -a gpurun_out/${TAG:-mm}_mmab.txt
  done
done
