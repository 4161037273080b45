#!/bin/bash
# A/B builds: recompile one source with extra defines and link it with the other in-tree objects
# into oaxaca-blinder-rs_amd/liboaxaca_boot_alt.so (load it with OB_LIB_PATH=... for timing runs).
# usage: bash tools/build_alt.sh ob_gram_i8.hip "-DOB_OZ_A_NT=0"
set -euo pipefail
SRC=$1; EXTRA=${2:-}
cd "$(dirname "$0")/../oaxaca-blinder-rs_amd/csrc"
make -s
mkdir -p ../build_alt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $EXTRA -c $SRC -o ../build_alt/$SRC.o
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../liboaxaca_boot_alt.so $OBJS ../build_alt/$SRC.o -lpthread -ldl
echo built ../liboaxaca_boot_alt.so with $SRC $EXTRA
