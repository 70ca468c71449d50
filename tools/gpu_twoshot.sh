# The fused two-shot launch: the multi-process tests that take it (DIRECT and
# SIGNAL, 2-8 PEs, and the unfused schedules), then tools/twoshot_probe.py at
# 2 and 4 PEs sharing the GPU, fused and unfused.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "signal_device_barriers or one_shot_unfused or all_pairs_sets_placements or eight_pe_baseline" \
    > gpurun_out/twoshot_tests.log 2>&1
rc=$?
tail -25 gpurun_out/twoshot_tests.log
[ $rc -eq 0 ] || exit $rc
probe() {   # npes, extra env
    timeout -k 10 180 env SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc $2 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node "$1" --master-addr 127.0.0.1 \
        --master-port 29517 tools/twoshot_probe.py
}
{ probe 2 "" && probe 2 SHMEMX_FUSED_TWOSHOT_KB=0 && probe 4 "" && probe 4 SHMEMX_FUSED_TWOSHOT_KB=0; } \
    > gpurun_out/twoshot_probe.txt 2> gpurun_out/twoshot_probe.err
rc=$?
cat gpurun_out/twoshot_probe.txt
[ $rc -eq 0 ] || tail -20 gpurun_out/twoshot_probe.err
exit $rc
