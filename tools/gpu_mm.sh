set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-mm}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --mm --cpu-seconds 0 > gpurun_out/${T}_bench_mm.json 2> gpurun_out/${T}_bench_mm.err && cat gpurun_out/${T}_bench_mm.json || { tail -20 gpurun_out/${T}_bench_mm.err; exit 1; }
