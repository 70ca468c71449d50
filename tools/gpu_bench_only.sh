# bench.py at N = 1, then the N > 1 code path rehearsed with 2 ranks on the
# one GPU (IPC transport).  Every GPU step has its own time limit; a failure
# ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; grep '"metric"' gpurun_out/bench.log | tail -1
[ $rc -eq 0 ] || exit $rc
SHMEMX_TRANSPORT=ipc SHMEMX_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/bench_rehearsal_n2.json 2> gpurun_out/bench_rehearsal_n2.err
rc=$?; echo "rehearsal rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_n2.json | tail -1
exit $rc
