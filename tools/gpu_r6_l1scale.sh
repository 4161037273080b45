set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in 64 128 256 512 1024 2048; do
  timeout -k 10 200 python bench.py --reps $R --cpu-seconds 0 --no-e2e --steps 20 --warmup 5 > gpurun_out/l1s_$R.json 2> gpurun_out/l1s_$R.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/l1s_$R.json').read().strip().splitlines()[-1]);print($R,{k:round(x,3) for k,x in d['breakdown_ms_per_step_rank0'].items()})"
done
