set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/bench3_$i.log 2>&1 || exit 1
  grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench3_$i.log
done
timeout -k 10 300 python bench.py --no-cpu-baseline --extras 0 --steps 400 --warmup 100 > gpurun_out/bench3_long.log 2>&1 || exit 1
grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench3_long.log
