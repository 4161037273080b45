#!/bin/bash
# One gpurun call: the -m gpu tests (optionally a -k filter) then a short default bench.
# usage: tools/gpu_check.sh [pytest -k expression] [tag]
set -o pipefail
K="${1:-}"
TAG="${2:-check}"
mkdir -p gpurun_out
ARGS=(-u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 900 python "${ARGS[@]}" > "gpurun_out/${TAG}_tests.log" 2>&1
rc=$?
tail -5 "gpurun_out/${TAG}_tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err"
rc=$?
tail -c 3000 "gpurun_out/${TAG}_bench.json"
[ $rc -ne 0 ] && exit $rc
if [ -n "${AB:-}" ] && [ -f oaxaca-blinder-rs_amd/liboaxaca_boot_alt.so ]; then  # A/B: the alternative build
  OB_LIB_PATH=$PWD/oaxaca-blinder-rs_amd/liboaxaca_boot_alt.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 \
    --cpu-seconds 0 --no-e2e > "gpurun_out/${TAG}_bench_alt.json" 2> "gpurun_out/${TAG}_bench_alt.err"
  rc=$?
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-e2e > "gpurun_out/${TAG}_bench_b.json" \
    2> "gpurun_out/${TAG}_bench_b.err" || exit $?
fi
exit $rc
