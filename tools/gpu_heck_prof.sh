set -o pipefail
# Heckman profile: f64 VALU PMC of ob_probit_kernel (-> profiles/pmc_probit.json, read by bench.py
# --heckman), a kernel-trace stats pass, then the bench itself; plus the configs[3] RIF line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
REPO=$PWD; OUT=$REPO/gpurun_out; T=${TAG:-hk}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
  --output-format csv -d "$OUT/${T}_pmc" -o run -- python3 "$REPO/bench.py" --heckman --steps 1 --warmup 0 --cpu-seconds 0 \
  > "$OUT/${T}_pmc.log" 2>&1 || { tail -5 "$OUT/${T}_pmc.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${T}_stats" -o run -- \
  python3 "$REPO/bench.py" --heckman --steps 2 --warmup 1 --cpu-seconds 0 > "$OUT/${T}_stats.log" 2>&1 || exit 1
cd "$REPO"
python tools/pmc_f64.py "$OUT/${T}_pmc" ob_probit_kernel "$OUT/${T}_pmc_probit.json" rows=1000000 preds=20 reps=2000 ks=4 || exit 1
cp "$OUT/${T}_pmc_probit.json" profiles/pmc_probit.json
timeout -k 10 300 python bench.py --heckman > "$OUT/${T}_bench_heckman.json" 2> "$OUT/${T}_bench_heckman.err" || { tail -5 "$OUT/${T}_bench_heckman.err"; exit 1; }
cat "$OUT/${T}_bench_heckman.json"
find "$OUT/${T}_stats" -name '*kernel_stats.csv' -exec head -8 {} \;
timeout -k 10 300 python bench.py --taus 0.1,0.5,0.9 --reps 5000 --cpu-seconds 0 > "$OUT/${T}_bench_rif3.json" 2> "$OUT/${T}_bench_rif3.err" && cat "$OUT/${T}_bench_rif3.json"
