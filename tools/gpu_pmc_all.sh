# Counters for every shipped kernel (tools/pmc_kernels.py): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in separate passes; summary -> gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 300 python3 tools/pmc_kernels.py > gpurun_out/pmc_kernels.log 2>&1 || { echo "plain run failed $?"; tail -5 gpurun_out/pmc_kernels.log; exit 1; }
cat gpurun_out/pmc_kernels.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pk_trace -o trace --output-format csv -- python3 tools/pmc_kernels.py > gpurun_out/pk_trace.log 2>&1 || { echo "trace failed $?"; tail -5 gpurun_out/pk_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pk_fetch -o fetch --output-format csv -- python3 tools/pmc_kernels.py > gpurun_out/pk_fetch.log 2>&1 || { echo "fetch failed $?"; tail -5 gpurun_out/pk_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pk_write -o write --output-format csv -- python3 tools/pmc_kernels.py > gpurun_out/pk_write.log 2>&1 || { echo "write failed $?"; tail -5 gpurun_out/pk_write.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/pmc_kernels.log gpurun_out/pk_trace gpurun_out/pk_fetch gpurun_out/pk_write gpurun_out/${TAG}_pmc_kernels.json > gpurun_out/pk_summary.txt 2>&1
cp gpurun_out/pk_trace/*kernel_stats.csv gpurun_out/${TAG}_pmc_kernels_stats.csv 2>/dev/null
find gpurun_out/pk_trace -name "*kernel_stats.csv" | head -2
cat gpurun_out/pk_summary.txt | head -150
