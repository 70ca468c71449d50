set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/sweep_fold32.py > gpurun_out/sweep32_$1.json 2> gpurun_out/sweep32.err; echo "rc=$?"
