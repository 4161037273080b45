set -o pipefail
# Effective clock + MFMA busy of oz_gram_kernel for OB_GRAM_DIAG 0 (full), 4 (no sub-tile loads), 2 (no MFMA).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-ck}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for d in 0 4 2; do
  OB_GRAM_DIAG=$d timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/${T}_d$d" -o run -- python3 "$R/tools/gram_ablate.py" > "$R/gpurun_out/${T}_d$d.log" 2>&1 || exit 1
  (cd "$R" && echo "diag $d" && python tools/pmc_clock.py gpurun_out/${T}_d$d oz_gram | tail -3 && python tools/pmc_kernel.py gpurun_out/${T}_d$d oz_gram_kernel)
done
