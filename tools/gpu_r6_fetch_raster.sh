#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the wide i8 Gram under its two rasters on one box (the in-tree library:
# contiguous groups per XCD; liboaxaca_boot_wr1.so: the chunk-major deal, tools/build_alt.sh
# ob_gram_i8.hip -DOB_OZ_W_RASTER=1 wr1). -> gpurun_out/TAG_raster.txt
set -euo pipefail
TAG=${1:-r6fr}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
B="python3 $REPO/bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e"
cd /tmp && export TMPDIR=/tmp
for V in base wr1; do
  if [ $V = wr1 ]; then export OB_LIB_PATH=$REPO/oaxaca-blinder-rs_amd/liboaxaca_boot_wr1.so; fi
  P=$OUT/${TAG}_$V
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${P}_fetch -o run -- $B > ${P}_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d ${P}_write -o run -- $B > ${P}_write.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d ${P}_tcc -o run -- $B > ${P}_tcc.log 2>&1
done
cd "$REPO"
S=$OUT/${TAG}_raster.txt
: > $S
for V in base wr1; do
  P=$OUT/${TAG}_$V
  echo "== $V" >> $S
  python tools/pmc_summary.py ${P}_fetch ${P}_write 1000000 20 10000 ${P}_pmc.json oz_gram_w_kernel >> $S
  python tools/pmc_clock.py ${P}_tcc oz_gram_w_kernel >> $S
done
cat $S
