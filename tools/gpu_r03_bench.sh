# Round 3: rocprofv3 passes over the N = 1 bench (tools/gpu_profile.sh), then
# the driver's default bench command on its own.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_profile.sh ${1:-r03} || exit $?
bash tools/gpu_pmc_all.sh ${1:-r03} || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?
cat gpurun_out/bench_n1.json
[ $rc -eq 0 ] || tail -20 gpurun_out/bench_n1.err
exit $rc
