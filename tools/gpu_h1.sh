set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_heckman.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/h1_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/h1_tests.log; exit 1; }
tail -1 gpurun_out/h1_tests.log
timeout -k 10 300 python bench.py --heckman --cpu-seconds 0 > gpurun_out/h1_heck.json 2> gpurun_out/h1_heck.err || { tail -20 gpurun_out/h1_heck.err; exit 1; }
timeout -k 10 120 python tools/gram_ablate.py > gpurun_out/h1_ab_nt.txt 2>&1 || exit 1
OB_LIB_PATH=$PWD/oaxaca-blinder-rs_amd/liboaxaca_boot_alt.so timeout -k 10 120 python tools/gram_ablate.py > gpurun_out/h1_ab_t.txt 2>&1 || exit 1
cat gpurun_out/h1_ab_nt.txt gpurun_out/h1_ab_t.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/h1_avail.txt 2>&1 || true
cd "$GRAFT_REPO_ROOT"
grep -i "F64\|FLOP" gpurun_out/h1_avail.txt | head -20 || true
