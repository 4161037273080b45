set -o pipefail
# A/B of the i8 Gram variants at the bench shape: tests, then bench (A in registers) and OB_OZ_AREG=0.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-ab}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram_i8.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in 1 0 1 0; do
  OB_OZ_AREG=$v timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/${T}_bench_areg$v.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python -c "import json,sys; j=json.load(open('gpurun_out/${T}_bench_areg$v.json')); print('areg=$v', round(j['value']), j['breakdown_ms_per_step_rank0'])"
done
for d in 0 2 4; do
  OB_GRAM_DIAG=$d timeout -k 10 120 python tools/gram_ablate.py 2>/dev/null | tee -a gpurun_out/${T}_ablate.txt || exit 1
done
