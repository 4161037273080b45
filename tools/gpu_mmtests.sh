set -o pipefail
# Machado-Mata GPU tests (parity with the oracle, the row reduction), then the configs[4] bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-mmt}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -22 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --mm --cpu-seconds 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
