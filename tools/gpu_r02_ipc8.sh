# Round 2, first GPU call: the P-input fold lab (warm / cold, real A2A shard
# size 4 Mi and 16 Mi per input), then the 8-PE multi-process tests (IPC
# DIRECT / GATHER / SIGNAL, configs[2] and configs[4] at 8 PEs, the RCCL test
# double at 8 ranks, 8-PE soaks) with the fence-coverage assertions.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "4194304 0" "4194304 1" "16777216 0" "16777216 1"; do
  timeout -k 10 120 ./tools/foldn_lab $a >> gpurun_out/foldn_lab.txt 2>&1 || { echo "lab failed $?"; tail -5 gpurun_out/foldn_lab.txt; exit 1; }
done
cat gpurun_out/foldn_lab.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_ipc.py -m gpu -x -v --timeout 900 --timeout-method thread \
  -k "${1:-8 or configs}" > gpurun_out/ipc8.log 2>&1
rc=$?; tail -40 gpurun_out/ipc8.log; exit $rc
