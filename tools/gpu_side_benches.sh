#!/bin/bash
# The non-headline bench lines at HEAD (configs[3] RIF multi-tau, Heckman, configs[4] Machado-Mata),
# one after another, each under its own time limit. -> gpurun_out/TAG_{rif3,heckman,mm}.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-side}
timeout -k 10 300 python bench.py --taus 0.1,0.5,0.9 --reps 5000 > gpurun_out/${TAG}_rif3.json 2> gpurun_out/${TAG}_rif3.err || exit $?
tail -c 600 gpurun_out/${TAG}_rif3.json; echo
timeout -k 10 300 python bench.py --heckman > gpurun_out/${TAG}_heckman.json 2> gpurun_out/${TAG}_heckman.err || exit $?
tail -c 600 gpurun_out/${TAG}_heckman.json; echo
timeout -k 10 400 python bench.py --mm > gpurun_out/${TAG}_mm.json 2> gpurun_out/${TAG}_mm.err || exit $?
tail -c 600 gpurun_out/${TAG}_mm.json; echo
