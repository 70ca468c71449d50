# Round 3 checkpoint: smoke(), the whole GPU suite, then the driver's default
# bench command (PE logs of the multi-process tests under gpurun_out/ipclogs).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_all.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?
cat gpurun_out/bench_n1.json
[ $rc -eq 0 ] || tail -20 gpurun_out/bench_n1.err
exit $rc
