#!/bin/bash
# Round-6 i8 Gram profile: the 8-wave kernel (gram_tile 1, oz_gram_kernel) against the wide-tile
# kernel (gram_tile 2, oz_gram_w_kernel) at configs[1], each with a kernel-trace stats pass and one
# rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE apart; the
# TCP block at most 4 counters). Uses the tuning library (it reads OB_GRAM_TILE). Run on the GPU box:
#   bash tools/gpu_r6_gramprof.sh TAG   -> gpurun_out/TAG_t{1,2}_*, summary gpurun_out/TAG_gram_pmc.txt
set -euo pipefail
TAG=${1:-r6gp}
OUT=$PWD/gpurun_out
REPO=$PWD
mkdir -p "$OUT"
export OB_LIB_PATH=$REPO/oaxaca-blinder-rs_amd/liboaxaca_boot_tuning.so
B="python3 $REPO/bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e"
cd /tmp && export TMPDIR=/tmp
for T in 1 2; do
  export OB_GRAM_TILE=$T
  P=$OUT/${TAG}_t$T
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d ${P}_stats -o run -- \
    python3 $REPO/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-e2e > ${P}_stats.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${P}_fetch -o run -- $B > ${P}_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d ${P}_write -o run -- $B > ${P}_write.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d ${P}_clock -o run -- $B > ${P}_clock.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    --output-format csv -d ${P}_tcp -o run -- $B > ${P}_tcp.log 2>&1
done
cd "$REPO"
S=$OUT/${TAG}_gram_pmc.txt
: > $S
for T in 1 2; do
  K=oz_gram_kernel; [ $T = 2 ] && K=oz_gram_w_kernel
  P=$OUT/${TAG}_t$T
  echo "== gram_tile $T ($K)" >> $S
  python tools/pmc_summary.py ${P}_fetch ${P}_write 1000000 20 10000 ${P}_pmc_gram.json $K >> $S
  python tools/pmc_clock.py ${P}_clock $K >> $S
  python tools/pmc_clock.py ${P}_tcp $K >> $S
  find ${P}_stats -name '*kernel_stats.csv' -exec grep -h "$K\|Name" {} \; >> $S
done
cat $S
