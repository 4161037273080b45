set -o pipefail
# count-kernel tiles-per-block A/B (liboaxaca_boot_ct{4,12,16}.so from tools/build_alt.sh ob_engine.hip -DOB_CNT_TILES=n)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for v in base ct4 ct12 ct16 base; do
  if [ $v = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
  env $E timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 20 --warmup 3 > gpurun_out/ct_$v.json 2> gpurun_out/ct_$v.err || { tail -20 gpurun_out/ct_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ct_$v.json'));print('$v',round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
