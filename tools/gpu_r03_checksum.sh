# Round 3: shmemx_checksum / verify per call vs the checksum grid cap, plus a
# kernel trace of each.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "4096 1" "2048 1" "2048 2"; do set -- $cfg; b=$1; export SHMEMX_CHECKSUM_UNROLL=$2; echo "unroll $2";
  SHMEMX_CHECKSUM_BLOCKS=$b timeout -k 10 120 python3 tools/checksum_probe.py > gpurun_out/ck_${b}_$2.log 2>&1 || { echo "probe $b failed"; tail -5 gpurun_out/ck_${b}_$2.log; exit 1; }
  grep blocks_cap gpurun_out/ck_${b}_$2.log
  SHMEMX_CHECKSUM_BLOCKS=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ck_trace_${b}_$2 -o trace --output-format csv -- python3 tools/checksum_probe.py > gpurun_out/ck_trace_${b}_$2.log 2>&1 || { echo "trace $b failed"; tail -5 gpurun_out/ck_trace_${b}_$2.log; exit 1; }
  grep -h checksum gpurun_out/ck_trace_${b}_$2/*kernel_stats.csv | cut -c1-200
done
