# Round 2: the randomized soak at 3/4 and 8 PEs on both transports, two
# seeds x 1000 calls (tests/gpu_ipc_child.py "soak"); PE logs under gpurun_out.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
for seed in ${SOAK_SEEDS:-21 22}; do
  SOAK_ITERS=1000 SOAK_SEED=$seed GPU_TEST_LOGDIR=gpurun_out/soak_logs_$seed timeout -k 10 560 \
    python -u -m pytest tests/test_gpu_ipc.py -k soak -x -v --timeout 540 --timeout-method thread \
    > gpurun_out/soak8_$seed.log 2>&1
  rc=$?; echo "seed $seed rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/soak8_$seed.log | tail -6
  [ $rc -eq 0 ] || exit $rc
done
