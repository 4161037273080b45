set -o pipefail
# Round-2 GPU script: gpu suite, smoke(), headline bench (plain and under torch.distributed.run at
# world 1), configs[2] strong mode. Each step under its own limit, chained so a failure stops it.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -3 gpurun_out/${T}_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo SMOKE_OK || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && cat gpurun_out/${T}_bench.json || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --cpu-seconds 0 > gpurun_out/${T}_bench_tr1.json 2> gpurun_out/${T}_bench_tr1.err && cat gpurun_out/${T}_bench_tr1.json || { tail -20 gpurun_out/${T}_bench_tr1.err; exit 1; }
timeout -k 10 300 python bench.py --strong --cpu-seconds 0 > gpurun_out/${T}_bench_strong.json 2> gpurun_out/${T}_bench_strong.err && cat gpurun_out/${T}_bench_strong.json
