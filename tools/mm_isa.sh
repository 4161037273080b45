#!/bin/bash
# Device ISA of the Machado-Mata kernels for one width (default K = 16) -> /tmp/mm_isa_K.s, plus
# per-kernel register / occupancy metadata. usage: bash tools/mm_isa.sh [K]
K=${1:-16}
cd "$(dirname "$0")/../oaxaca-blinder-rs_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DOB_MM_ISA_K=$K $EXTRA --cuda-device-only -S ob_mm.hip -o /tmp/mm_isa_$K.s
grep -E "^\s+\.(name|vgpr_count|agpr_count|sgpr_count|group_segment_fixed_size|private_segment_fixed_size):" /tmp/mm_isa_$K.s | grep -B1 -A5 "mm_" | head -80
