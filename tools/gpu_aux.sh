set -o pipefail
# Side-config benches with their CPU baselines (Heckman, Machado-Mata configs[4], RIF configs[3])
# plus the Heckman kernel-trace profile. Each step under its own limit; a failure ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-aux}
timeout -k 10 400 python bench.py --heckman > gpurun_out/${T}_heckman.json 2> gpurun_out/${T}_heckman.err && cat gpurun_out/${T}_heckman.json || { tail -20 gpurun_out/${T}_heckman.err; exit 1; }
timeout -k 10 500 python bench.py --mm > gpurun_out/${T}_mm.json 2> gpurun_out/${T}_mm.err && cat gpurun_out/${T}_mm.json || { tail -20 gpurun_out/${T}_mm.err; exit 1; }
timeout -k 10 300 python bench.py --taus 0.1,0.5,0.9 --reps 5000 > gpurun_out/${T}_rif3.json 2> gpurun_out/${T}_rif3.err && cat gpurun_out/${T}_rif3.json || { tail -20 gpurun_out/${T}_rif3.err; exit 1; }
bash tools/profile_heckman.sh ${T} > gpurun_out/${T}_hkprof.log 2>&1 && tail -30 gpurun_out/${T}_hkprof.log
