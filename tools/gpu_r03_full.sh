# Round 3: the whole GPU suite (PE logs of the multi-process tests kept under
# gpurun_out/ipclogs), then the driver's default bench command.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ulimit -c 0
export GPU_TEST_LOGDIR=gpurun_out/ipclogs
# the job's CPU share and, every 30 s, the busiest processes (multi-PE tests
# run 8 PE processes at once)
{ echo "affinity: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') CPUs, nproc $(nproc)";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/cpu.txt
( while true; do date +%T; ps -eo pid,ppid,pcpu,etime,rss,args --sort=-pcpu | head -15 | cut -c1-160; sleep 30; done ) > gpurun_out/ps.log 2>&1 &
MON=$!
trap 'kill $MON 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_all.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?
cat gpurun_out/bench_n1.json
[ $rc -eq 0 ] || tail -20 gpurun_out/bench_n1.err
exit $rc
