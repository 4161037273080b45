#!/bin/bash
# Timing A/B of environment switches on the in-tree library: one short bench per setting, the
# settings in order and then again (A B A B), optional parity tests under the last setting first.
# usage: TAG=x TESTS="tests/test_gpu_gram_i8.py" bash tools/ab_env.sh "" "OB_OZ_WAVES=4" ...
#   BENCH_ARGS="--mm" times another workload (default: configs[1])
#   (an empty string is the default environment) -> gpurun_out/TAG_env<i>_<round>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
source "$(dirname "${BASH_SOURCE[0]}")/tuning_env.sh"  # OB_* switches: tuning build only
T=${TAG:-abenv}
if [ -n "${TESTS:-}" ]; then
  for e in "$@"; do
    [ -z "$e" ] && continue
    env $e timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > "gpurun_out/${T}_tests.log" 2>&1 || { tail -40 "gpurun_out/${T}_tests.log"; exit 1; }
    echo "tests under [$e]: $(tail -1 gpurun_out/${T}_tests.log)"
  done
fi
for r in 1 2; do
  i=0
  for e in "$@"; do
    out="gpurun_out/${T}_env${i}_${r}.json"
    env $e timeout -k 10 300 python bench.py --cpu-seconds 0 --no-e2e ${BENCH_ARGS:-} --steps ${STEPS:-10} --warmup 3 \
      > "$out" 2> "${out%.json}.err" || { tail -20 "${out%.json}.err"; exit 1; }
    python -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);b=d.get('breakdown_ms_per_step_rank0') or {k:v for k,v in d['roofline'].items() if k.endswith('_ms')};print('[$e]',round(d['value'],2),{k:round(v,3) for k,v in b.items()})"
    i=$((i+1))
  done
done
