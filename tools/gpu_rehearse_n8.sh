# The driver's N = 4 and N = 8 bench command rehearsed on the one GPU
# (numbers never reported: 8 processes share one GPU): IPC transport with
# every extra, then the default RCCL transport through the RCCL test double
# (headline only at 8 ranks, every extra at 4; its rates are the double's
# host-memory shim).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export SHMEMX_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2
for n in 4 8; do
  SHMEMX_TRANSPORT=ipc timeout -k 10 560 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 5 --warmup 2 \
    > gpurun_out/rehearse_ipc_n$n.json 2> gpurun_out/rehearse_ipc_n$n.err
  rc=$?; echo "ipc n=$n rc=$rc"; grep '"metric"' gpurun_out/rehearse_ipc_n$n.json | tail -1 | cut -c1-600
  [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_ipc_n$n.err; exit $rc; }
done
export FAKE_RCCL=$GRAFT_REPO_ROOT/tests/native/libfake_rccl.so FAKE_RCCL_BOX_KB=16384
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 8 --steps 3 --warmup 1 --extras 0 \
  > gpurun_out/rehearse_rccl_n8.json 2> gpurun_out/rehearse_rccl_n8.err
rc=$?; echo "rccl double n=8 rc=$rc"; grep '"metric"' gpurun_out/rehearse_rccl_n8.json | tail -1 | cut -c1-600
[ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_rccl_n8.err; exit $rc; }
# every extra on the RCCL transport at 4 ranks (smaller nreduce: the double
# moves data through host memory)
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --gpus 4 --steps 3 --warmup 1 --nreduce 1048576 \
  > gpurun_out/rehearse_rccl_n4_extras.json 2> gpurun_out/rehearse_rccl_n4_extras.err
rc=$?; echo "rccl double n=4 extras rc=$rc"
[ $rc -eq 0 ] || tail -20 gpurun_out/rehearse_rccl_n4_extras.err
exit $rc
