set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 ./tools/fold_lab 33554432 ${1:-0} > gpurun_out/lab_${1:-0}.txt 2>&1; echo "rc=$?"
