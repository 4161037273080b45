set -o pipefail
# level-1/count kernel check: bitwise count tests, then the headline bench twice (level-1 timing)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-l1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 20 --warmup 3 > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || { tail -20 gpurun_out/${T}_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_bench$i.json'));print(round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
