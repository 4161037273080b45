# Sourced by the A/B scripts that set OB_* environment switches: those are read only by the tuning
# build (make -C oaxaca-blinder-rs_amd/csrc tuning -> liboaxaca_boot_tuning.so; ob_options.hpp).
_T=${GRAFT_REPO_ROOT:-$PWD}/oaxaca-blinder-rs_amd/liboaxaca_boot_tuning.so
if [ ! -f "$_T" ]; then
  echo "tools: $_T is missing; build it with: make -C oaxaca-blinder-rs_amd/csrc tuning" >&2
  exit 1
fi
export OB_LIB_PATH=${OB_LIB_PATH:-$_T}
