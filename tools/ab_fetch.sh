#!/bin/bash
# HBM read bytes of one kernel for the in-tree library ("base") and alternative builds
# (tools/build_alt.sh ... NAME): one rocprofv3 FETCH_SIZE pass each over a one-step bench.
#   usage: [KERNEL=oz_gram_kernel] [BENCH_ARGS=...] TAG=x bash tools/ab_fetch.sh NAME...
#   -> gpurun_out/TAG_fetch_NAME/, summary lines (2 x FETCH_SIZE per dispatch, GB) on stdout
set -o pipefail
REPO=$PWD
OUT=$REPO/gpurun_out
L=$REPO/oaxaca-blinder-rs_amd
K=${KERNEL:-oz_gram_kernel}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  if [ "$v" = base ]; then unset OB_LIB_PATH; else export OB_LIB_PATH=$L/liboaxaca_boot_$v.so; fi
  d="$OUT/${TAG:-ab}_fetch_$v"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d" -o run -- \
    python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --no-e2e ${BENCH_ARGS:-} > "$d.log" 2>&1 \
    || { tail -20 "$d.log"; exit 1; }
  python3 - "$d" "$K" "$v" <<'EOF'
import csv, glob, os, sys
d, k, v = sys.argv[1:4]
vals = {}
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        if k in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
gb = [2.0 * x * 1024 / 1e9 for x in vals.values()]
print(v, k, "read GB per dispatch (2 x FETCH_SIZE):", [round(x, 2) for x in gb])
EOF
done
unset OB_LIB_PATH
