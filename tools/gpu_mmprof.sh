set -o pipefail
# rocprofv3 kernel stats of the Machado-Mata bench (configs[4]) -> gpurun_out/${TAG}_mmprof/
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-mmp}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_mmprof -o run -- python3 bench.py --mm --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/${T}_mmprof.json 2> gpurun_out/${T}_mmprof.err || { tail -20 gpurun_out/${T}_mmprof.err; exit 1; }
cat gpurun_out/${T}_mmprof.json | head -c 300; echo
f=$(find gpurun_out/${T}_mmprof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -30
