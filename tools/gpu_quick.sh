set -o pipefail
# quick GPU check: i8 Gram tests, a parity slice, then the headline bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram_i8.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && cat gpurun_out/${T}_bench.json || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
