set -o pipefail
# A/B of the Machado-Mata variants at configs[4]: OB_MM_IL (state layout) x OB_MM_PC (assemble form)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-mab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in "1 0" "1 1" "0 0"; do
  set -- $v
  OB_MM_IL=$1 OB_MM_PC=$2 timeout -k 10 300 python bench.py --mm --cpu-seconds 0 --steps 3 > gpurun_out/${T}_il$1_pc$2.json 2>> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  python -c "import json; j=json.load(open('gpurun_out/${T}_il$1_pc$2.json')); r=j['roofline']; print('il=$1 pc=$2', round(j['value'],3), 'reps/s assemble_ms', round(r['assemble_ms'],1), 'GB/s', round(r['achieved']))"
done
