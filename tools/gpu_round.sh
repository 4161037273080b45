set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1_gputests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r1_gputests.log; exit 1; }
tail -3 gpurun_out/r1_gputests.log
timeout -k 10 300 python bench.py > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err && cat gpurun_out/r1_bench.json
timeout -k 10 300 python bench.py --mm > gpurun_out/r1_bench_mm.json 2> gpurun_out/r1_bench_mm.err && cat gpurun_out/r1_bench_mm.json
