set -o pipefail
# full GPU suite, smoke, then the headline bench twice at the driver's step counts
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-f2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -1 gpurun_out/${T}_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $([ $i = 2 ] && echo --cpu-seconds 0) > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || { tail -20 gpurun_out/${T}_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_bench$i.json'));print(round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
