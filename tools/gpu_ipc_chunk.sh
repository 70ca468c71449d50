set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ipc.py -k chunks -m gpu -x -q --capture=sys > gpurun_out/ipc_chunk.log 2>&1
rc=$?; tail -60 gpurun_out/ipc_chunk.log; exit $rc
