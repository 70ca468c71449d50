# The peers fold (all inputs' loads in flight: DIRECT's and SIGNAL's fold
# phase) and the segment-interleaved gather: fold fuzz through both kernels,
# the IPC tests that run DIRECT / SIGNAL, then the local-HBM rate of both
# fold kernels (tools/fold_n_probe.py).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
timeout -k 10 700 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_fold.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "fuzz or signal_device_barriers or one_shot_unfused or all_pairs_sets_placements or eight_pe_baseline or staged_in_chunks or soak or full_size" \
    > gpurun_out/peers_tests.log 2>&1
rc=$?
tail -30 gpurun_out/peers_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/fold_n_probe.py > gpurun_out/foldn_peers_probe.txt 2>&1
rc=$?
cat gpurun_out/foldn_peers_probe.txt
exit $rc
