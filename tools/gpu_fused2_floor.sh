# The fused launches' own time with no peer to wait for: 1 PE with the
# collective schedules forced (SHMEMX_FORCE_COLLECTIVE=1), DIRECT and SIGNAL
# at one-shot (8 B, 64 KiB) and two-shot (512 KiB ... 4 MiB) sizes, under
# rocprofv3 --kernel-trace --stats, for each grid size in $FUSED_BLOCKS_LIST
# ($SHMEMX_FUSED_BLOCKS).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp SHMEMX_FORCE_COLLECTIVE=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
export PROBE_KIB=0.0078125,64,512,1024,2048,4096
for fb in ${FUSED_BLOCKS_LIST:-64}; do
  SHMEMX_FUSED_BLOCKS=$fb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fused_prof_$fb -o trace \
    --output-format csv -- python3 tools/twoshot_probe.py > gpurun_out/fused_floor_$fb.txt 2>&1 \
    || { echo "failed $?"; tail -20 gpurun_out/fused_floor_$fb.txt; exit 1; }
  echo "blocks $fb: $(grep fused_twoshot_kb gpurun_out/fused_floor_$fb.txt)"
  f=$(find gpurun_out/fused_prof_$fb -name "*kernel_stats.csv" | head -1)
  grep -E "signal_fold" "$f" | cut -d, -f1-4 | sed "s/^/blocks $fb: /"
done
