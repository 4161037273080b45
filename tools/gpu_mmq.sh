set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
OB_MM_TRACE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_mm.py -m gpu -x -v --timeout 300 --timeout-method thread -k "reduction" > gpurun_out/mmq_tests.log 2>&1 || { echo TESTS_FAILED; grep -v "^\[mm\] iteration" gpurun_out/mmq_tests.log | tail -60; exit 1; }
grep -v "^\[mm\] iteration" gpurun_out/mmq_tests.log | tail -30
