# Round 3: small-call latency breakdown, then the whole GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
timeout -k 10 120 ./tools/latency_breakdown > gpurun_out/latency_breakdown.txt 2>&1 || { echo "latency probe failed $?"; tail -5 gpurun_out/latency_breakdown.txt; exit 1; }
cat gpurun_out/latency_breakdown.txt
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_all.log | head -20; tail -40 gpurun_out/gpu_all.log; }
exit $rc
