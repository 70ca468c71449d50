set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_ipc.py tests/test_gpu_collectives.py tests/test_gpu_api.py -m gpu -x -q --capture=sys > gpurun_out/ipc_tests.log 2>&1
rc=$?; tail -30 gpurun_out/ipc_tests.log; [ $rc -eq 0 ] || exit $rc
# rehearsal of bench.py's N > 1 path: 2 ranks sharing the GPU, IPC transport
SHMEMX_TRANSPORT=ipc SHMEMX_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/bench_rehearsal_n2.json 2> gpurun_out/bench_rehearsal_n2.err
rc=$?; cat gpurun_out/bench_rehearsal_n2.json; tail -5 gpurun_out/bench_rehearsal_n2.err; exit $rc
