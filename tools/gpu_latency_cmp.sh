# Small-call latency (tools/pe_latency_probe.py): 1 PE with the collective
# schedules forced, then 2 PEs sharing the GPU over the IPC transport.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 \
          --master-addr 127.0.0.1 --master-port $1 tools/pe_latency_probe.py; }
SHMEMX_FORCE_COLLECTIVE=1 SHMEMX_TRANSPORT=ipc PROBE_STEPS=${PROBE_STEPS:-none} \
  run 29531 1 > gpurun_out/pelat_1pe.txt 2> gpurun_out/pelat_1pe.err || { tail -5 gpurun_out/pelat_1pe.err; exit 1; }
echo "1 PE:"; grep after gpurun_out/pelat_1pe.txt
SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc PROBE_STEPS=${PROBE_STEPS:-none} \
  run 29532 2 > gpurun_out/pelat_2pe.txt 2> gpurun_out/pelat_2pe.err || { tail -5 gpurun_out/pelat_2pe.err; exit 1; }
echo "2 PEs:"; grep after gpurun_out/pelat_2pe.txt
