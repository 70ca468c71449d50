# Round 3: the cold mid-size fold (tools/cold_midsize_probe.py): timings,
# then a kernel trace and FETCH_SIZE / WRITE_SIZE in separate rocprofv3 passes.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/cold_midsize_probe.py 10 > gpurun_out/cold_probe.log 2>&1 || { echo "plain run failed $?"; tail -5 gpurun_out/cold_probe.log; exit 1; }
cat gpurun_out/cold_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cm_trace -o trace --output-format csv -- python3 tools/cold_midsize_probe.py 5 > gpurun_out/cm_trace.log 2>&1 || { echo "trace failed $?"; tail -5 gpurun_out/cm_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cm_fetch -o fetch --output-format csv -- python3 tools/cold_midsize_probe.py 5 > gpurun_out/cm_fetch.log 2>&1 || { echo "fetch failed $?"; tail -5 gpurun_out/cm_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/cm_write -o write --output-format csv -- python3 tools/cold_midsize_probe.py 5 > gpurun_out/cm_write.log 2>&1 || { echo "write failed $?"; tail -5 gpurun_out/cm_write.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/cm_trace.log gpurun_out/cm_trace gpurun_out/cm_fetch gpurun_out/cm_write gpurun_out/r03_cold_midsize_pmc.json > gpurun_out/cm_summary.txt 2>&1
grep -E '"config"|traffic_over_alg|rocprof_avg_us' gpurun_out/cm_summary.txt | head -80
