# GPU round trip: pytest -m gpu, then bench.py (N=1).  Every GPU step has its
# own time limit; a crash/abort/timeout ends the script (no further GPU work).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --capture=sys > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; grep '"metric"' gpurun_out/bench.log | tail -1
[ $rc -eq 0 ] || exit $rc
# rehearsal of the N > 1 bench path: 2 ranks sharing the GPU, IPC transport
SHMEMX_TRANSPORT=ipc SHMEMX_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/bench_rehearsal_n2.json 2> gpurun_out/bench_rehearsal_n2.err
rc=$?; echo "rehearsal rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_n2.json | tail -1
exit $rc
