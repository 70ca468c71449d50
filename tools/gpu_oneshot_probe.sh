# Small-call latency of DIRECT and SIGNAL (the fused one shot and the small
# two shot), 2 and 8 PE processes sharing the GPU: tools/twoshot_probe.py at
# 8 B ... 1 MiB per PE.  $1 names the output file.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-oneshot}
export SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc PROBE_KIB=0.0078125,8,64,256,1024
for n in 2 8; do
  [ $n -gt 4 ] && export GPU_MAX_HW_QUEUES=2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2954$n tools/twoshot_probe.py >> gpurun_out/$tag.txt 2>> gpurun_out/$tag.err || exit $?
done
cat gpurun_out/$tag.txt
