set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --capture=sys > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/bench3_$i.log 2>&1 || exit 1
  grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench3_$i.log
done
timeout -k 10 300 python tools/fold_lab 2>/dev/null; timeout -k 10 300 ./tools/fold_lab 33554432 0 | head -2
