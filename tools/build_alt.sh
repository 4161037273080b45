#!/bin/bash
# A/B builds: recompile one source with extra defines and link it with the other in-tree objects
# into oaxaca-blinder-rs_amd/liboaxaca_boot_NAME.so (default NAME alt; load it with OB_LIB_PATH=...
# for timing runs, tools/ab_libs.sh). usage: bash tools/build_alt.sh ob_gram_i8.hip "-DOB_OZ_A_NT=0" [NAME]
set -euo pipefail
SRC=$1; EXTRA=${2:-}; NAME=${3:-alt}
cd "$(dirname "$0")/../oaxaca-blinder-rs_amd/csrc"
make -s
mkdir -p ../build_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $EXTRA -c $SRC -o ../build_$NAME/$SRC.o
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../liboaxaca_boot_$NAME.so $OBJS ../build_$NAME/$SRC.o -lpthread -ldl
echo built ../liboaxaca_boot_$NAME.so with $SRC $EXTRA
