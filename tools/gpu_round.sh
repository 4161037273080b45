set -o pipefail
# Round GPU script: the gpu test suite, smoke(), then the headline, RIF, Machado-Mata and Heckman
# bench lines; each step under its own time limit, chained so a failure stops the run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1_gputests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r1_gputests.log; exit 1; }
tail -2 gpurun_out/r1_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 && echo SMOKE_OK || { tail -20 gpurun_out/r1_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err && cat gpurun_out/r1_bench.json || exit 1
timeout -k 10 300 python bench.py --taus 0.1,0.5,0.9 --reps 5000 > gpurun_out/r1_bench_rif3.json 2> gpurun_out/r1_bench_rif3.err && cat gpurun_out/r1_bench_rif3.json || exit 1
timeout -k 10 300 python bench.py --mm > gpurun_out/r1_bench_mm.json 2> gpurun_out/r1_bench_mm.err && cat gpurun_out/r1_bench_mm.json || exit 1
timeout -k 10 300 python bench.py --heckman > gpurun_out/r1_bench_heckman.json 2> gpurun_out/r1_bench_heckman.err && cat gpurun_out/r1_bench_heckman.json
