# Round 3: peers/gather lab, the kernel timing list (verify included), then
# the cold mid-size probe with its rocprofv3 passes.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/peers_gather_lab > gpurun_out/peers_gather_lab.txt 2>&1 || { echo "lab failed $?"; tail -5 gpurun_out/peers_gather_lab.txt; exit 1; }
cat gpurun_out/peers_gather_lab.txt
timeout -k 10 200 python3 tools/pmc_kernels.py > gpurun_out/pk_quick.log 2>&1 || { echo "pmc_kernels failed $?"; tail -5 gpurun_out/pk_quick.log; exit 1; }
cat gpurun_out/pk_quick.log
bash tools/gpu_r03_cold.sh
