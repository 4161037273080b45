set -o pipefail
# count-kernel change: full GPU suite, headline bench, and the 8-GPU strong share (1250 reps) on one GPU
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-cnt}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -2 gpurun_out/${T}_gputests.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && cat gpurun_out/${T}_bench.json || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 --reps 1250 --steps 20 --warmup 2 > gpurun_out/${T}_bench1250.json 2> gpurun_out/${T}_bench1250.err && cat gpurun_out/${T}_bench1250.json || { tail -20 gpurun_out/${T}_bench1250.err; exit 1; }
