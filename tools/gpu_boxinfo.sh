set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
(rocm-smi --showmemorypartition --showcomputepartition 2>/dev/null | grep -iE "partition|GPU\[" | head -6) || true
(rocm-smi --showclocks 2>/dev/null | grep -E "mclk|fclk|socclk|sclk" | head -6) || true
timeout -k 10 300 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/benchbox.log 2>&1 || exit 1
grep -o '"avg_launch_us": [0-9.]*' gpurun_out/benchbox.log
timeout -k 10 300 ./tools/fold_lab 33554432 0 | head -1
