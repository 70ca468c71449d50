set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/sweep_fold.py > gpurun_out/sweep.json 2> gpurun_out/sweep.err; echo "sweep rc=$?"
tail -12 gpurun_out/sweep.json
