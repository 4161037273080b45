#!/bin/bash
# Round 5: two sub-tiles per barrier (liboaxaca_boot_sub2.so) -- parity on the Gram/parity tests,
# then timing against the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh sub2 tests/test_gpu_gram_i8.py tests/test_gpu_parity.py || exit 1
TAG=sub2b bash tools/ab_libs.sh sub2
