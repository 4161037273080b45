#!/bin/bash
# Round 5, Gram raster A/B: parity of the in-tree build (chunk-major raster) on the Gram/parity
# GPU tests, then timing and HBM reads against the round-4 raster (liboaxaca_boot_r0.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_gram_i8.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5r_tests.log 2>&1 \
  || { tail -40 gpurun_out/r5r_tests.log; exit 1; }
tail -2 gpurun_out/r5r_tests.log
TAG=r5r bash tools/ab_libs.sh r0 r0 || exit 1
TAG=r5r bash tools/ab_fetch.sh r0
