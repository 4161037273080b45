#!/bin/bash
# Round-end evidence on one GPU box (run from the repo root): the GPU suite, smoke(), the driver's
# bench form, the round profile (tools/profile_round.sh), the bench under torch.distributed.run at
# world 1, configs[2]'s per-GPU share, and the --gpus 2 refusal on a one-GPU box.
#   bash tools/round_end.sh TAG   -> gpurun_out/TAG_*
set -o pipefail
TAG=${1:-rXX_head}
O=gpurun_out
mkdir -p $O
step() { echo "[round_end] $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/${TAG}_gputests.txt 2>&1 || { tail -30 $O/${TAG}_gputests.txt; exit 1; }
tail -1 $O/${TAG}_gputests.txt
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.txt 2>&1 \
  || { tail -30 $O/${TAG}_smoke.txt; exit 1; }
tail -1 $O/${TAG}_smoke.txt
step bench
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err \
  || { tail -30 $O/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]);print(round(d['value']),d['roofline']['frac'],d['breakdown_ms_per_step_rank0'])"
step profile
SKIP_BENCH=1 bash tools/profile_round.sh $TAG > $O/${TAG}_profile.log 2>&1 || { tail -30 $O/${TAG}_profile.log; exit 1; }
head -c 1500 $O/${TAG}_profile.log
step torchrun1
timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/${TAG}_torchrun1.json 2> $O/${TAG}_torchrun1.err \
  || { tail -30 $O/${TAG}_torchrun1.err; exit 1; }
step share1250
timeout -k 10 400 python bench.py --reps 1250 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e \
  > $O/${TAG}_share1250.json 2> $O/${TAG}_share1250.err || { tail -30 $O/${TAG}_share1250.err; exit 1; }
step gpus2
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > $O/${TAG}_gpus2.out 2> $O/${TAG}_gpus2.err
echo "bench.py --gpus 2 on this box: exit $? ($(tail -1 $O/${TAG}_gpus2.err))" | tee $O/${TAG}_gpus2.txt
step done
