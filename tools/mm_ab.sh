set -o pipefail
# A/B of Machado-Mata kernel variants: env settings in $VARIANTS (space-separated NAME=VALUE or "base");
# per variant the bench value and the per-kernel times of a rocprofv3 kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  rm -rf gpurun_out/ab_$v
  if [ "$v" = base ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$v -o run -- python3 bench.py --mm --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  echo "== $v: $(python3 -c "import json;print(round(json.load(open('gpurun_out/ab_$v.json'))['value'],3))") replicates/s"
  python3 tools/mm_trace_split.py $(find gpurun_out/ab_$v -name "*kernel_trace.csv" | head -1) | head -8
done
