# rocprofv3 passes over the 1-GPU bench: kernel trace + stats, then FETCH_SIZE
# and WRITE_SIZE in separate --pmc passes; summarised into profiles/.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
# the kernel trace is of the driver's own command (bench.py with its defaults);
# the PMC passes skip the extras and the CPU baseline (counter collection
# serialises every launch)
B="--steps 20 --warmup 5 --no-cpu-baseline --extras 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- python3 bench.py > gpurun_out/prof_trace.log 2>&1 || { echo "trace failed $?"; tail -5 gpurun_out/prof_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch --output-format csv -- python3 bench.py $B > gpurun_out/prof_fetch.log 2>&1 || { echo "fetch failed $?"; tail -5 gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write --output-format csv -- python3 bench.py $B > gpurun_out/prof_write.log 2>&1 || { echo "write failed $?"; tail -5 gpurun_out/prof_write.log; exit 1; }
python3 tools/summarize_prof.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write $TAG > gpurun_out/prof_summary.json 2>&1
cp profiles/${TAG}_* gpurun_out/ 2>/dev/null
grep -h '"metric"' gpurun_out/prof_trace.log | head -1
cat gpurun_out/prof_summary.json | head -60
