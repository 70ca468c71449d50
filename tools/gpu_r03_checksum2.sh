# Round 3: checksum finish on the device (last workgroup) vs on the host
# (per-workgroup slots in page-locked memory), per call and per kernel.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for f in device host device host; do
  SHMEMX_CHECKSUM_FINISH=$f timeout -k 10 120 python3 tools/checksum_probe.py > gpurun_out/ck2_$f.log 2>&1 || { echo "probe $f failed"; tail -5 gpurun_out/ck2_$f.log; exit 1; }
  echo "$f: $(grep blocks_cap gpurun_out/ck2_$f.log)"
done
for f in device host; do
  SHMEMX_CHECKSUM_FINISH=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ck2_trace_$f -o trace --output-format csv -- python3 tools/checksum_probe.py > gpurun_out/ck2_trace_$f.log 2>&1 || { echo "trace $f failed"; exit 1; }
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/ck2_trace_$f/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'checksum' in r['Name']: print('$f kernel', r['Name'][:70], 'avg', round(float(r['AverageNs'])/1e3,2), 'us min', round(float(r['MinNs'])/1e3,2))"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_checksum.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
SHMEMX_CHECKSUM_FINISH=device timeout -k 10 300 python -u -m pytest tests/test_gpu_checksum.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
