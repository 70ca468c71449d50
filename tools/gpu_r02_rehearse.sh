# Round 2: the N > 1 bench path rehearsed on the one GPU (numbers never
# reported): 2 ranks over the IPC transport, then 2 ranks on the default RCCL
# transport through the RCCL test double.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SHMEMX_TRANSPORT=ipc SHMEMX_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/bench_rehearsal_ipc_n2.json 2> gpurun_out/bench_rehearsal_ipc_n2.err
rc=$?; echo "ipc rehearsal rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_ipc_n2.json | tail -1 | cut -c1-1500
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_rehearsal_ipc_n2.err; exit $rc; }
bash tools/gpu_rehearse_rccl.sh
