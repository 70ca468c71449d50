# GPU round trip: pytest -m gpu, then bench.py (N=1).  Every GPU step has its
# own time limit; a crash/abort/timeout ends the script (no further GPU work).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --capture=sys > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; grep '"metric"' gpurun_out/bench.log | tail -1
exit $rc
