#!/bin/bash
# Clock and MFMA busy of the wide Gram under timing ablations (tuning build): one rocprofv3 --pmc pass
# per gram_diag value at configs[1]. usage: bash tools/gpu_r6_diag_clock.sh TAG DIAG...
set -euo pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
export OB_LIB_PATH=$REPO/oaxaca-blinder-rs_amd/liboaxaca_boot_tuning.so
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  export OB_GRAM_DIAG=$d
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $OUT/${TAG}_d$d -o run -- python3 $REPO/bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e \
    > $OUT/${TAG}_d$d.log 2>&1
  echo "gram_diag $d: $(cd $REPO && python tools/pmc_clock.py $OUT/${TAG}_d$d oz_gram_w_kernel | tail -1)" | tee -a $OUT/${TAG}_diag_clock.txt
done
