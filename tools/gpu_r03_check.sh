# Round 3: kernel timings (tools/pmc_kernels.py), then the whole GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
timeout -k 10 200 python3 tools/pmc_kernels.py > gpurun_out/pk_quick.log 2>&1 || { echo "pmc_kernels failed $?"; tail -5 gpurun_out/pk_quick.log; exit 1; }
grep config gpurun_out/pk_quick.log
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_all.log | head -20; tail -40 gpurun_out/gpu_all.log; }
exit $rc
