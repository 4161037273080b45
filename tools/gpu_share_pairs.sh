#!/bin/bash
# configs[2]'s per-GPU share (1,250 replicates) against the configs[1] line (10,000) on one box, in
# alternating pairs, so the share ratio is read off the same box and hour.
#   bash tools/gpu_share_pairs.sh TAG [PAIRS]   -> gpurun_out/TAG_pairs.txt (+ each JSON line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-r6pairs}; P=${2:-3}
OUT=gpurun_out/${T}_pairs.txt
: > $OUT
summ() {
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['value']),round(d['ms_per_step'],4),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})" "$1" "$2"
}
for i in $(seq 1 $P); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e \
    > gpurun_out/${T}_bench_$i.json 2> gpurun_out/${T}_bench_$i.err || { tail -30 gpurun_out/${T}_bench_$i.err; exit 1; }
  summ gpurun_out/${T}_bench_$i.json "10k#$i" | tee -a $OUT
  timeout -k 10 300 python bench.py --reps 1250 --steps 40 --warmup 5 --cpu-seconds 0 --no-e2e \
    > gpurun_out/${T}_share_$i.json 2> gpurun_out/${T}_share_$i.err || { tail -30 gpurun_out/${T}_share_$i.err; exit 1; }
  summ gpurun_out/${T}_share_$i.json "1250#$i" | tee -a $OUT
done
python - "$T" "$P" <<'EOF' | tee -a $OUT
import json, sys
t, p = sys.argv[1], int(sys.argv[2])
v = lambda f: json.loads(open(f).read().strip().splitlines()[-1])["value"]
b = [v(f"gpurun_out/{t}_bench_{i}.json") for i in range(1, p + 1)]
s = [v(f"gpurun_out/{t}_share_{i}.json") for i in range(1, p + 1)]
print("ratio per pair", [round(y / x, 4) for x, y in zip(b, s)], "mean", round(sum(s) / sum(b), 4))
EOF
