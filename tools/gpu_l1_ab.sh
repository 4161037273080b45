#!/bin/bash
# Level-1 kernel A/B between two source trees (the in-tree one and a copy of another commit built
# under DIR, e.g. _ab_old/): a short bench each for the timing, then two SQ counter passes each.
# usage: bash tools/gpu_l1_ab.sh TAG DIR   -> gpurun_out/TAG_l1ab_*.txt
set -euo pipefail
TAG=${1:-l1ab}
ALT=${2:-_ab_old}
REPO=$PWD
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
for side in new old; do
  if [ $side = new ]; then T=$REPO; else T=$REPO/$ALT; fi
  (cd "$T" && timeout -k 10 300 python bench.py --cpu-seconds 0 --no-e2e --steps 10 --warmup 3) \
    > "$OUT/${TAG}_$side.json" 2> "$OUT/${TAG}_$side.err"
  python -c "import json;d=json.loads(open('$OUT/${TAG}_$side.json').read().strip().splitlines()[-1]);print('$side',round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
cd /tmp && export TMPDIR=/tmp
for side in new old; do
  if [ $side = new ]; then T=$REPO; else T=$REPO/$ALT; fi
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/${TAG}_${side}_p$i" -o run -- \
      python3 "$T/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e > "$OUT/${TAG}_${side}_p$i.log" 2>&1
    (cd "$REPO" && python tools/pmc_clock.py "$OUT/${TAG}_${side}_p$i" ob_level1_kernel | tail -1 | sed "s/^/$side p$i /") \
      | tee -a "$OUT/${TAG}_l1ab.txt"
    i=$((i+1))
  done
done
