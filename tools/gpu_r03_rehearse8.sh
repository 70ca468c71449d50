# Round 3: the driver's N = 8 bench command (full sizes, every extra) rehearsed
# on the one GPU over the IPC transport (8 processes share it: rates never
# reported), timed, to see the extras finish inside the watchdog and carry
# xgmi_links / auto_recommendation.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export SHMEMX_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2
start=$SECONDS
SHMEMX_TRANSPORT=ipc timeout -k 10 700 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29528 bench.py --gpus 8 --steps 5 --warmup 2 \
  > gpurun_out/rehearse8_ipc.json 2> gpurun_out/rehearse8_ipc.err
rc=$?
echo "ipc n=8 rc=$rc wall_s=$((SECONDS - start))"
grep '"metric"' gpurun_out/rehearse8_ipc.json | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
e = d['extras']
print('correct', d['correct'], 'note', e.get('note'))
print('xgmi_links', json.dumps(e.get('xgmi_links'))[:600])
print('auto_recommendation env', json.dumps((e.get('auto_recommendation') or {}).get('env')))
print('extras', sorted(e))
"
[ $rc -eq 0 ] || tail -20 gpurun_out/rehearse8_ipc.err
exit $rc
