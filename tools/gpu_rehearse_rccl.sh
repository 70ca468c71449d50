# The N > 1 bench path on the default RCCL transport, rehearsed with 2 ranks
# on the one GPU through the RCCL test double (numbers meaningless: host-memory
# shim).  Headline only first, then with every extra at a smaller nreduce.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export FAKE_RCCL=$GRAFT_REPO_ROOT/tests/native/libfake_rccl.so SHMEMX_SHARE_GPU=1 FAKE_RCCL_BOX_KB=16384
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --extras 0 \
  > gpurun_out/rehearse_rccl.json 2> gpurun_out/rehearse_rccl.err
rc=$?; echo "headline rc=$rc"; grep '"metric"' gpurun_out/rehearse_rccl.json | tail -1 | cut -c1-900
[ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_rccl.err; exit $rc; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29514 bench.py --gpus 2 --steps 3 --warmup 1 --nreduce 1048576 \
  > gpurun_out/rehearse_rccl_extras.json 2> gpurun_out/rehearse_rccl_extras.err
rc=$?; echo "extras rc=$rc"; grep '"metric"' gpurun_out/rehearse_rccl_extras.json | tail -1
[ $rc -eq 0 ] || tail -20 gpurun_out/rehearse_rccl_extras.err
exit $rc
