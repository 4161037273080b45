set -o pipefail
# level-1 A/B: the in-tree build against bitop3 Philox builds (liboaxaca_boot_l1u{2,3,4}.so, tools/build_alt.sh
# ob_engine.hip "-DOB_L1_X3 -DOB_L1_UNROLL=u"), headline bench per variant, counts tests on each variant
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/oaxaca-blinder-rs_amd
for v in base l1u2 l1u3 l1u4 base; do
  if [ $v = base ]; then E=""; else E="OB_LIB_PATH=$L/liboaxaca_boot_$v.so"; fi
  env $E timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 20 --warmup 3 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v',round(d['value']),{k:round(v,3) for k,v in d['breakdown_ms_per_step_rank0'].items()})"
done
for v in l1u2 l1u3 l1u4; do
  OB_LIB_PATH=$L/liboaxaca_boot_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q -k counts --timeout 120 --timeout-method thread > gpurun_out/ab_${v}_tests.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/ab_${v}_tests.log; exit 1; }
  echo $v $(tail -1 gpurun_out/ab_${v}_tests.log)
done
