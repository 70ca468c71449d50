# Round 3: selected GPU tests (pytest -k expression in $1), PE logs kept
# under gpurun_out/ipclogs.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 ${2:-900} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$1" > gpurun_out/sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/sel.log | tail -40
[ $rc -eq 0 ] || tail -60 gpurun_out/sel.log
exit $rc
