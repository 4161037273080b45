#!/bin/bash
# A/B of an alternative build NAME (tools/build_alt.sh): its parity on the resample/Gram/parity GPU
# tests first, then tools/ab_libs.sh timing against the in-tree library.
#   usage: bash tools/gpu_ab_lib.sh NAME [pytest files...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
NAME=$1; shift
FILES=${*:-tests/test_gpu_multi.py tests/test_gpu_gram_i8.py tests/test_gpu_parity.py}
L=$PWD/oaxaca-blinder-rs_amd
OB_LIB_PATH=$L/liboaxaca_boot_$NAME.so timeout -k 10 500 python -u -m pytest $FILES -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${NAME}_tests.log 2>&1 || { tail -40 gpurun_out/${NAME}_tests.log; exit 1; }
tail -2 gpurun_out/${NAME}_tests.log
TAG=$NAME bash tools/ab_libs.sh $NAME
