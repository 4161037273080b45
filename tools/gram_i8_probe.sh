set -o pipefail
# Ablations (OB_GRAM_DIAG 0/2/4/6) and an SQ stall-counter pass of oz_gram_kernel at the bench shape.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-p}
for d in 0 2 4 6; do
  OB_GRAM_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py >> gpurun_out/${T}_ablate.txt 2>&1 || exit 1
done
cat gpurun_out/${T}_ablate.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_sq" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/${T}_sq.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python tools/pmc_kernel.py gpurun_out/${T}_sq oz_gram_kernel
