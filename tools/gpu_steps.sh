# The one GPU runner: `gpurun -- bash tools/gpu_steps.sh STEP [STEP ...]`.
# Each step runs under its own time limit and writes under gpurun_out/; the
# first step that fails (a test failure, a crash, an abort, a time limit)
# ends the script, so nothing more touches the GPU after trouble.
#
#   smoke          __graft_entry__.smoke()
#   tests          pytest -m gpu (the whole GPU suite; PE logs in gpurun_out/ipclogs)
#   tests_k        the GPU tests matching $TESTS_K (pytest -k)
#   bench          the driver's default command, python bench.py (N = 1)
#   bench2         the same again (run-to-run check of value and cpu_baseline)
#   trace          rocprofv3 --kernel-trace --stats of the driver's command, python3 bench.py
#   pmc            FETCH_SIZE and WRITE_SIZE of the headline, one rocprofv3 pass each, then
#                  tools/summarize_prof.py -> gpurun_out/profiles/$TAG_{kernel_stats.csv,pmc.json}
#   pmc_kernels    every shipped kernel (tools/pmc_kernels.py): trace + FETCH/WRITE passes
#   soak           the randomized multi-PE soak (tests/gpu_ipc_child.py "soak"),
#                  $SOAK_SEEDS x $SOAK_ITERS draws
#   isx_mirror     tools/isx_mirror_latency.py, plain and with the collective schedule forced
#   mirror_cost    tools/mirror_cost_probe: page-protection changes and block flushes
# $TAG names the round's files (default r06).
#   small_calls    tools/small_call_probe.py plain and under rocprofv3 (1 PE; IPC / RCCL collective schedule forced)
#   ceiling        tools/stream_lab: copy / read / fill ceilings beside the fold
#   write          tools/stream_lab: write-only shapes (what bounds the fold's stores)
#   fold2, copy2, gs  tools/stream_lab: fold / copy shapes the write-only lab suggests
#   copy           tools/copy_probe.py under a rocprofv3 kernel trace: the library's copy kernel
#   rehearse2      bench.py N = 2 on the IPC transport, both ranks on this GPU
#   rehearse8      the same with 8 ranks
#   rehearse_rccl  bench.py N = $REH_N (2) on the RCCL transport against the RCCL test double
#                  (extras capped at $REH_EXTRAS_MAX elements: the double moves every byte through host memory)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out

run() {   # run <seconds> <log> <cmd...>: one GPU step under its own limit
    local secs=$1 log=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $* -> rc=$rc"
    [ $rc -eq 0 ] || { tail -25 "$log"; exit $rc; }
}

json_line() {   # json_line <log> <json>: the bench line alone, as a JSON file
    grep '^{"metric"' "$1" > "$2" && cut -c1-400 "$2"
}

BENCH_HEAD="python3 bench.py --steps 20 --warmup 5 --extras 0 --no-cpu-baseline"
TAG=${TAG:-r06}

for step in "$@"; do
    case $step in
    smoke) run 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()"; tail -2 $O/smoke.log ;;
    tests)
        export GPU_TEST_LOGDIR=$O/ipclogs
        run 1100 $O/gpu_tests.log python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread
        tail -3 $O/gpu_tests.log ;;
    tests_k)   # a subset: TESTS_K="expr" (pytest -k)
        export GPU_TEST_LOGDIR=$O/ipclogs
        run 900 $O/gpu_tests_k.log python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$TESTS_K"
        tail -3 $O/gpu_tests_k.log ;;
    bench|bench2)   # the log keeps rank 0's progress lines; the .json holds the one bench line
        b=bench_n1; [ $step = bench2 ] && b=bench_n1_b
        run 600 $O/$b.log python3 bench.py; json_line $O/$b.log $O/$b.json ;;
    trace)
        run 600 $O/trace.log rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py
        grep '"metric"' $O/trace.log | cut -c1-300
        python3 tools/trace_by_grid.py $O/trace fold > $O/trace_by_grid.txt; cat $O/trace_by_grid.txt ;;
    pmc)
        run 200 $O/pmc_fetch.log timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- $BENCH_HEAD
        run 200 $O/pmc_write.log timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- $BENCH_HEAD
        PROFILES_OUT=$O/profiles python3 tools/summarize_prof.py $O/trace $O/pmc_fetch $O/pmc_write $TAG > $O/prof_summary.json 2>&1
        head -40 $O/prof_summary.json ;;
    pmc_kernels)
        run 300 $O/pmc_kernels.log python3 tools/pmc_kernels.py
        run 300 $O/pk_trace.log rocprofv3 --kernel-trace --stats -d $O/pk_trace -o trace --output-format csv -- python3 tools/pmc_kernels.py
        run 320 $O/pk_fetch.log timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pk_fetch -o fetch --output-format csv -- python3 tools/pmc_kernels.py
        run 320 $O/pk_write.log timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pk_write -o write --output-format csv -- python3 tools/pmc_kernels.py
        python3 tools/summarize_pmc.py $O/pmc_kernels.log $O/pk_trace $O/pk_fetch $O/pk_write $O/${TAG}_pmc_kernels.json > $O/pk_summary.txt 2>&1
        cp $O/pk_trace/*/*kernel_stats.csv $O/${TAG}_pmc_kernels_stats.csv 2>/dev/null || cp $O/pk_trace/*kernel_stats.csv $O/${TAG}_pmc_kernels_stats.csv
        head -80 $O/pk_summary.txt ;;
    soak)
        for seed in ${SOAK_SEEDS:-51}; do
            SOAK_ITERS=${SOAK_ITERS:-1000} SOAK_SEED=$seed GPU_TEST_LOGDIR=$O/soak_logs_$seed run 600 $O/soak_$seed.log \
                python3 -u -m pytest tests/test_gpu_ipc.py -k soak -x -v --timeout 580 --timeout-method thread
            grep -E "PASSED|FAILED|passed|failed" $O/soak_$seed.log | tail -6
        done ;;
    isx_mirror)
        run 120 $O/isx_mirror.json python3 tools/isx_mirror_latency.py 3000
        SHMEMX_FORCE_COLLECTIVE=1 run 120 $O/isx_mirror_coll.json python3 tools/isx_mirror_latency.py 2000
        cat $O/isx_mirror*.json ;;
    small_calls)   # configs[0]'s call at n 1/1024/4096, heap and host operands, wall (C timer) and kernel time
        for mode in plain ipc_coll rccl_coll; do
            envs=""; [ $mode = ipc_coll ] && envs="SHMEMX_TRANSPORT=ipc SHMEMX_FORCE_COLLECTIVE=1"
            [ $mode = rccl_coll ] && envs="SHMEMX_FORCE_COLLECTIVE=1"
            env $envs timeout -k 10 120 python3 tools/small_call_probe.py 3000 > $O/small_calls_$mode.json 2>$O/small_calls_$mode.err \
                || { tail -20 $O/small_calls_$mode.err; exit 1; }
            cat $O/small_calls_$mode.json
            ([ -n "$envs" ] && export $envs; run 200 $O/small_calls_${mode}_trace.log rocprofv3 --kernel-trace --stats -d $O/small_calls_${mode}_trace \
                -o t --output-format csv -- python3 tools/small_call_probe.py 3000)
            cp $O/small_calls_${mode}_trace/*kernel_stats.csv $O/small_calls_${mode}_kernel_stats.csv 2>/dev/null \
                || cp $O/small_calls_${mode}_trace/*/*kernel_stats.csv $O/small_calls_${mode}_kernel_stats.csv
            cut -d, -f1-5 $O/small_calls_${mode}_kernel_stats.csv | cut -c1-220
        done ;;
    mirror_cost) run 120 $O/mirror_cost.txt ./tools/mirror_cost_probe 2000; cat $O/mirror_cost.txt ;;
    ceiling)
        for nd in 33554432 67108864; do
            run 300 $O/stream_lab_ceiling_$nd.txt ./tools/stream_lab $nd 3 10 ceiling
            cut -c1-260 $O/stream_lab_ceiling_$nd.txt
        done ;;
    write|fold2|copy2|gs)
        for nd in 33554432 67108864; do
            run 300 $O/stream_lab_${step}_$nd.txt ./tools/stream_lab $nd 3 10 $step
            cut -c1-260 $O/stream_lab_${step}_$nd.txt
        done ;;
    copy)
        run 300 $O/copy_probe.txt rocprofv3 --kernel-trace --stats -d $O/copy_probe -o t --output-format csv \
            -- python3 tools/copy_probe.py
        grep copy $O/copy_probe.txt; python3 tools/trace_by_grid.py $O/copy_probe fold_kernel ;;
    rehearse2|rehearse8)
        np=${step#rehearse}
        q=4; [ "$np" -gt 4 ] && q=2     # 8 processes' queues on one GPU (tests/test_gpu_ipc.py)
        GPU_MAX_HW_QUEUES=$q SHMEMX_TRANSPORT=ipc SHMEMX_SHARE_GPU=1 run 900 $O/rehearse_ipc_n$np.log python3 -m torch.distributed.run \
            --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $np \
            --steps 10 --warmup 3
        json_line $O/rehearse_ipc_n$np.log $O/rehearse_ipc_n$np.json ;;
    rehearse_rccl)   # $REH_N ranks (default 2)
        np=${REH_N:-2}; q=4; [ "$np" -gt 4 ] && q=2
        GPU_MAX_HW_QUEUES=$q FAKE_RCCL=$PWD/tests/native/libfake_rccl.so SHMEMX_SHARE_GPU=1 run 900 $O/rehearse_rccl_n$np.log \
            python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
            --master-port 29512 bench.py --gpus $np --steps 10 --warmup 3 --extras-max-nreduce ${REH_EXTRAS_MAX:-1048576}
        json_line $O/rehearse_rccl_n$np.log $O/rehearse_rccl_n$np.json ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
