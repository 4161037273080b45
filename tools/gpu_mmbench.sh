set -o pipefail
# Machado-Mata bench (configs[4]) with the row reduction (default) and without (OB_MM_REDUCE=0)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-mmb}
OB_MM_TRACE=1 timeout -k 10 300 python bench.py --mm --cpu-seconds 0 > gpurun_out/${T}_on.json 2> gpurun_out/${T}_on.err || { tail -30 gpurun_out/${T}_on.err; exit 1; }
cat gpurun_out/${T}_on.json
grep -v "iteration" gpurun_out/${T}_on.err | tail -30
OB_MM_REDUCE=0 timeout -k 10 300 python bench.py --mm --cpu-seconds 0 > gpurun_out/${T}_off.json 2> gpurun_out/${T}_off.err || { tail -30 gpurun_out/${T}_off.err; exit 1; }
cat gpurun_out/${T}_off.json
