set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/sweep_cold.py > gpurun_out/sweep_cold.json 2> gpurun_out/sweep_cold.err; echo "rc=$?"
